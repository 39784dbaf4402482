// amd-smi session: see smi.h. Only the header's types are used at compile time
// (KGS_HAVE_AMDSMI); every function is resolved with dlsym, so a missing symbol
// degrades that one query instead of failing the load.
#include "smi.h"

#include <dlfcn.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#ifdef KGS_HAVE_AMDSMI
#include <amd_smi/amdsmi.h>
#endif

namespace kgs {
namespace gpuinfo {

#ifdef KGS_HAVE_AMDSMI

struct SmiSession::Api {
  decltype(&amdsmi_init) init = nullptr;
  decltype(&amdsmi_shut_down) shut_down = nullptr;
  decltype(&amdsmi_get_socket_handles) sockets = nullptr;
  decltype(&amdsmi_get_processor_handles) procs = nullptr;
  decltype(&amdsmi_get_gpu_enumeration_info) enum_info = nullptr;
  decltype(&amdsmi_get_gpu_device_bdf) bdf = nullptr;
  decltype(&amdsmi_get_gpu_device_uuid) uuid = nullptr;
  decltype(&amdsmi_get_gpu_total_ecc_count) ecc = nullptr;
  decltype(&amdsmi_get_gpu_xgmi_link_status) xgmi_status = nullptr;
  decltype(&amdsmi_topo_get_link_type) link_type = nullptr;
  decltype(&amdsmi_topo_get_link_weight) link_weight = nullptr;
  decltype(&amdsmi_is_P2P_accessible) p2p = nullptr;
  bool initialized = false;
};

std::unique_ptr<SmiSession> SmiSession::open() {
  if (std::getenv("KGS_NO_AMDSMI")) return nullptr;
  std::unique_ptr<SmiSession> s(new SmiSession());
  s->api_.reset(new Api());
  const char* over = std::getenv("KGS_AMDSMI_LIB");
  const char* names[] = {over, "libamd_smi.so", "libamd_smi.so.26", "/opt/rocm/lib/libamd_smi.so"};
  for (const char* n : names) {
    if (!n || !*n) continue;
    s->dl_ = ::dlopen(n, RTLD_NOW | RTLD_LOCAL);
    if (s->dl_) {
      s->lib_ = n;
      break;
    }
    if (over && n == over) return nullptr;  // an explicit library that does not load: no silent fallback
  }
  if (!s->dl_) return nullptr;
  Api& a = *s->api_;
#define KGS_SYM(f, n) a.f = reinterpret_cast<decltype(a.f)>(::dlsym(s->dl_, n))
  KGS_SYM(init, "amdsmi_init");
  KGS_SYM(shut_down, "amdsmi_shut_down");
  KGS_SYM(sockets, "amdsmi_get_socket_handles");
  KGS_SYM(procs, "amdsmi_get_processor_handles");
  KGS_SYM(enum_info, "amdsmi_get_gpu_enumeration_info");
  KGS_SYM(bdf, "amdsmi_get_gpu_device_bdf");
  KGS_SYM(uuid, "amdsmi_get_gpu_device_uuid");
  KGS_SYM(ecc, "amdsmi_get_gpu_total_ecc_count");
  KGS_SYM(xgmi_status, "amdsmi_get_gpu_xgmi_link_status");
  KGS_SYM(link_type, "amdsmi_topo_get_link_type");
  KGS_SYM(link_weight, "amdsmi_topo_get_link_weight");
  KGS_SYM(p2p, "amdsmi_is_P2P_accessible");
#undef KGS_SYM
  if (!a.init || !a.shut_down || !a.sockets || !a.procs) return nullptr;
  if (a.init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return nullptr;
  a.initialized = true;
  uint32_t nsock = 0;
  if (a.sockets(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS || nsock == 0) return s;  // no GPUs: empty session
  std::vector<amdsmi_socket_handle> socks(nsock);
  a.sockets(&nsock, socks.data());
  for (auto sk : socks) {
    uint32_t np = 0;
    if (a.procs(sk, &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
    std::vector<amdsmi_processor_handle> ps(np);
    a.procs(sk, &np, ps.data());
    for (auto p : ps) {
      SmiGpu g;
      g.handle = p;
      if (a.enum_info) {
        amdsmi_enumeration_info_t ei{};
        if (a.enum_info(p, &ei) == AMDSMI_STATUS_SUCCESS) g.render_minor = (int)ei.drm_render;
      }
      if (a.bdf) {
        amdsmi_bdf_t b{};
        if (a.bdf(p, &b) == AMDSMI_STATUS_SUCCESS) {
          char buf[32];
          std::snprintf(buf, sizeof buf, "%04x:%02x:%02x.%x", (unsigned)b.domain_number, (unsigned)b.bus_number,
                        (unsigned)b.device_number, (unsigned)b.function_number);
          g.bdf = buf;
        }
      }
      if (a.uuid) {
        char u[AMDSMI_MAX_STRING_LENGTH] = {0};
        unsigned len = sizeof u;
        if (a.uuid(p, &len, u) == AMDSMI_STATUS_SUCCESS) g.uuid = u;
      }
      s->gpus_.push_back(g);
    }
  }
  return s;
}

SmiSession::~SmiSession() {
  if (api_ && api_->initialized && api_->shut_down) api_->shut_down();
  if (dl_) ::dlclose(dl_);
}

bool SmiSession::health(const SmiGpu& g, SmiHealth& out) const {
  const Api& a = *api_;
  out = SmiHealth();
  if (a.ecc) {
    amdsmi_error_count_t ec{};
    if (a.ecc((amdsmi_processor_handle)g.handle, &ec) == AMDSMI_STATUS_SUCCESS) {
      out.ecc_ok = true;
      out.ecc_correctable = (int64_t)ec.correctable_count;
      out.ecc_uncorrectable = (int64_t)ec.uncorrectable_count;
      out.ecc_deferred = (int64_t)ec.deferred_count;
    }
  }
  if (a.xgmi_status) {
    amdsmi_xgmi_link_status_t ls{};
    if (a.xgmi_status((amdsmi_processor_handle)g.handle, &ls) == AMDSMI_STATUS_SUCCESS) {
      out.links_ok = true;
      const int n = (int)(ls.total_links < AMDSMI_MAX_NUM_XGMI_LINKS ? ls.total_links : AMDSMI_MAX_NUM_XGMI_LINKS);
      out.links_total = n;
      out.links_up = out.links_down = 0;
      for (int i = 0; i < n; ++i) {
        const int st = ls.status[i] == AMDSMI_XGMI_LINK_UP ? 1 : ls.status[i] == AMDSMI_XGMI_LINK_DOWN ? 0 : 2;
        out.link_state.push_back(st);
        out.links_up += st == 1;
        out.links_down += st == 0;
      }
    }
  }
  return out.ecc_ok || out.links_ok;
}

SmiLink SmiSession::link(const SmiGpu& x, const SmiGpu& y) const {
  const Api& a = *api_;
  SmiLink L;
  if (a.link_type) {
    uint64_t hops = 0;
    amdsmi_link_type_t t = AMDSMI_LINK_TYPE_UNKNOWN;
    if (a.link_type((amdsmi_processor_handle)x.handle, (amdsmi_processor_handle)y.handle, &hops, &t) ==
        AMDSMI_STATUS_SUCCESS) {
      L.ok = true;
      L.hops = hops;
      L.type = t == AMDSMI_LINK_TYPE_XGMI ? 11 : t == AMDSMI_LINK_TYPE_PCIE ? 2 : 0;
    }
  }
  if (a.link_weight) {
    uint64_t w = 0;
    if (a.link_weight((amdsmi_processor_handle)x.handle, (amdsmi_processor_handle)y.handle, &w) ==
        AMDSMI_STATUS_SUCCESS)
      L.weight = w;
  }
  if (a.p2p) {
    bool acc = false;
    if (a.p2p((amdsmi_processor_handle)x.handle, (amdsmi_processor_handle)y.handle, &acc) == AMDSMI_STATUS_SUCCESS)
      L.p2p = acc ? 1 : 0;
  }
  return L;
}

#else  // built without the amd-smi header: the session never opens

struct SmiSession::Api {};
std::unique_ptr<SmiSession> SmiSession::open() { return nullptr; }
SmiSession::~SmiSession() {}
bool SmiSession::health(const SmiGpu&, SmiHealth& out) const {
  out = SmiHealth();
  return false;
}
SmiLink SmiSession::link(const SmiGpu&, const SmiGpu&) const { return SmiLink(); }

#endif

const SmiGpu* SmiSession::by_minor(int minor) const {
  for (auto& g : gpus_)
    if (minor >= 0 && g.render_minor == minor) return &g;
  return nullptr;
}

const SmiGpu* SmiSession::by_bdf(const std::string& bdf) const {
  for (auto& g : gpus_)
    if (!bdf.empty() && g.bdf == bdf) return &g;
  return nullptr;
}

}  // namespace gpuinfo
}  // namespace kgs
