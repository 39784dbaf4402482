// kgs gpuinfo core: KFD sysfs topology parser + optional amd-smi enrichment.
// See gpuinfo.h for the model. C++17, no ROCm link-time dependency: amd-smi is
// dlopen'ed so the device-plugin image does not need ROCm installed.
#include "gpuinfo.h"

#include <dirent.h>
#include <dlfcn.h>
#include <sys/stat.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>

#ifdef KGS_HAVE_AMDSMI
#include <amd_smi/amdsmi.h>
#endif

namespace kgs {
namespace gpuinfo {

namespace {

std::string join(const std::string& root, const std::string& path) {
  if (root.empty() || root == "/") return path;
  std::string r = root;
  while (r.size() > 1 && r.back() == '/') r.pop_back();
  return r + path;
}

bool exists(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0;
}

bool read_file(const std::string& p, std::string& out) {
  std::ifstream f(p);
  if (!f) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return true;
}

std::map<std::string, std::string> read_props(const std::string& p, bool* ok) {
  std::map<std::string, std::string> m;
  std::string s;
  *ok = read_file(p, s) && !s.empty();
  std::istringstream is(s);
  std::string line;
  while (std::getline(is, line)) {
    auto sp = line.find(' ');
    if (sp == std::string::npos) continue;
    m[line.substr(0, sp)] = line.substr(sp + 1);
  }
  return m;
}

uint64_t u64(const std::map<std::string, std::string>& m, const char* k, uint64_t d = 0) {
  auto it = m.find(k);
  if (it == m.end()) return d;
  try {
    return std::stoull(it->second);
  } catch (...) {
    return d;
  }
}

std::vector<std::string> list_dir(const std::string& p) {
  std::vector<std::string> out;
  DIR* d = ::opendir(p.c_str());
  if (!d) return out;
  while (auto* e = ::readdir(d)) {
    if (e->d_name[0] == '.') continue;
    out.emplace_back(e->d_name);
  }
  ::closedir(d);
  return out;
}

std::vector<int> numeric_entries(const std::string& p) {
  std::vector<int> ids;
  for (auto& n : list_dir(p)) {
    char* end = nullptr;
    long v = std::strtol(n.c_str(), &end, 10);
    if (end && *end == '\0') ids.push_back((int)v);
  }
  std::sort(ids.begin(), ids.end());
  return ids;
}

std::string bdf_from(uint64_t domain, uint64_t location) {
  // KFD location_id = (bus << 8) | (device << 3) | function
  char buf[32];
  std::snprintf(buf, sizeof buf, "%04x:%02x:%02x.%x", (unsigned)domain, (unsigned)((location >> 8) & 0xff),
                (unsigned)((location >> 3) & 0x1f), (unsigned)(location & 0x7));
  return buf;
}

int read_int_file(const std::string& p, int d) {
  std::string s;
  if (!read_file(p, s)) return d;
  try {
    return std::stoi(s);
  } catch (...) {
    return d;
  }
}

std::string json_escape(const std::string& s) {
  std::string o;
  for (char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      default:
        if ((unsigned char)c < 0x20) {
          char b[8];
          std::snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o += c;
        }
    }
  }
  return o;
}

// ---- amd-smi (optional) ------------------------------------------------------
#ifdef KGS_HAVE_AMDSMI
struct Smi {
  void* h = nullptr;
  decltype(&amdsmi_init) init = nullptr;
  decltype(&amdsmi_shut_down) shut_down = nullptr;
  decltype(&amdsmi_get_socket_handles) sockets = nullptr;
  decltype(&amdsmi_get_processor_handles) procs = nullptr;
  decltype(&amdsmi_get_gpu_enumeration_info) enum_info = nullptr;
  decltype(&amdsmi_get_gpu_device_bdf) bdf = nullptr;
  decltype(&amdsmi_get_gpu_device_uuid) uuid = nullptr;

  bool load() {
    for (const char* name : {"libamd_smi.so", "libamd_smi.so.26", "/opt/rocm/lib/libamd_smi.so"}) {
      h = ::dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) return false;
#define KGS_SYM(f, n) f = reinterpret_cast<decltype(f)>(::dlsym(h, n))
    KGS_SYM(init, "amdsmi_init");
    KGS_SYM(shut_down, "amdsmi_shut_down");
    KGS_SYM(sockets, "amdsmi_get_socket_handles");
    KGS_SYM(procs, "amdsmi_get_processor_handles");
    KGS_SYM(enum_info, "amdsmi_get_gpu_enumeration_info");
    KGS_SYM(bdf, "amdsmi_get_gpu_device_bdf");
    KGS_SYM(uuid, "amdsmi_get_gpu_device_uuid");
#undef KGS_SYM
    return init && shut_down && sockets && procs;
  }
  ~Smi() {
    if (h) ::dlclose(h);
  }
};

bool enrich_with_amdsmi(Topology& t) {
  if (std::getenv("KGS_NO_AMDSMI")) return false;
  Smi s;
  if (!s.load()) return false;
  if (s.init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return false;
  uint32_t nsock = 0;
  if (s.sockets(&nsock, nullptr) != AMDSMI_STATUS_SUCCESS || nsock == 0) {
    s.shut_down();
    return false;
  }
  std::vector<amdsmi_socket_handle> socks(nsock);
  s.sockets(&nsock, socks.data());
  bool any = false;
  for (auto sk : socks) {
    uint32_t np = 0;
    if (s.procs(sk, &np, nullptr) != AMDSMI_STATUS_SUCCESS || np == 0) continue;
    std::vector<amdsmi_processor_handle> ps(np);
    s.procs(sk, &np, ps.data());
    for (auto p : ps) {
      int minor = -1;
      std::string bdf;
      if (s.enum_info) {
        amdsmi_enumeration_info_t ei{};
        if (s.enum_info(p, &ei) == AMDSMI_STATUS_SUCCESS) minor = (int)ei.drm_render;
      }
      if (s.bdf) {
        amdsmi_bdf_t b{};
        if (s.bdf(p, &b) == AMDSMI_STATUS_SUCCESS) {
          char buf[32];
          std::snprintf(buf, sizeof buf, "%04x:%02x:%02x.%x", (unsigned)b.domain_number, (unsigned)b.bus_number,
                        (unsigned)b.device_number, (unsigned)b.function_number);
          bdf = buf;
        }
      }
      char uuid[AMDSMI_MAX_STRING_LENGTH] = {0};
      unsigned len = sizeof uuid;
      std::string u;
      if (s.uuid && s.uuid(p, &len, uuid) == AMDSMI_STATUS_SUCCESS) u = uuid;
      for (auto& g : t.gpus) {
        if ((minor >= 0 && g.render_minor == minor) || (!bdf.empty() && g.bdf == bdf)) {
          if (!u.empty()) g.uuid = u;
          any = true;
        }
      }
    }
  }
  s.shut_down();
  return any;
}
#else
bool enrich_with_amdsmi(Topology&) { return false; }
#endif

}  // namespace

std::string gfx_name(uint32_t v) {
  if (!v) return "";
  unsigned major = v / 10000, minor = (v / 100) % 100, step = v % 100;
  char buf[32];
  std::snprintf(buf, sizeof buf, "gfx%u%x%x", major, minor, step);
  return buf;
}

bool refresh_health(const std::string& root, Gpu& g) {
  const std::string kfd = join(root, "/dev/kfd");
  const std::string rnode = join(root, "/dev/dri/renderD" + std::to_string(g.render_minor));
  const std::string props = join(root, "/sys/class/kfd/kfd/topology/nodes/" + std::to_string(g.node_id) + "/properties");
  g.render_node_present = g.render_minor >= 0 && exists(rnode);
  bool ok = false;
  auto m = read_props(props, &ok);
  if (!exists(kfd)) {
    g.healthy = false;
    g.health_reason = "/dev/kfd missing";
  } else if (!g.render_node_present) {
    g.healthy = false;
    g.health_reason = "render node " + rnode + " missing";
  } else if (!ok) {
    // A cgroup-restricted node reads empty although the device works; only a
    // KFD node that disappeared entirely counts as lost.
    g.healthy = exists(props);
    g.health_reason = g.healthy ? "ok (topology properties not readable here)" : "KFD node gone";
  } else if (u64(m, "simd_count") == 0) {
    g.healthy = false;
    g.health_reason = "KFD node reports no SIMDs";
  } else {
    g.healthy = true;
    g.health_reason = "ok";
  }
  return g.healthy;
}

Topology discover(const std::string& root, bool use_amdsmi) {
  Topology t;
  t.root = root.empty() ? "/" : root;
  const std::string topo = join(root, "/sys/class/kfd/kfd/topology/nodes");
  t.kfd_present = exists(join(root, "/dev/kfd"));
  t.topology_present = exists(topo);
  if (!t.topology_present) {
    t.warnings.push_back("no KFD topology at " + topo);
    return t;
  }
  std::vector<int> render_nodes;
  for (auto& n : list_dir(join(root, "/dev/dri"))) {
    if (n.rfind("renderD", 0) == 0) render_nodes.push_back(std::atoi(n.c_str() + 7));
  }
  std::sort(render_nodes.begin(), render_nodes.end());

  for (int id : numeric_entries(topo)) {
    const std::string nd = topo + "/" + std::to_string(id);
    bool ok = false;
    auto m = read_props(nd + "/properties", &ok);
    Gpu g;
    g.node_id = id;
    g.properties_readable = ok;
    if (ok) {
      if (u64(m, "simd_count") == 0) {  // CPU node
        t.cpu_nodes++;
        continue;
      }
      g.render_minor = (int)u64(m, "drm_render_minor", (uint64_t)-1);
      g.gfx_target_version = (uint32_t)u64(m, "gfx_target_version");
      g.gfx_arch = gfx_name(g.gfx_target_version);
      g.vendor_id = (uint32_t)u64(m, "vendor_id");
      g.device_id = (uint32_t)u64(m, "device_id");
      g.simd_count = (int)u64(m, "simd_count");
      const int spc = (int)u64(m, "simd_per_cu", 4);
      g.cu_count = spc ? g.simd_count / spc : 0;
      g.num_xcc = (int)u64(m, "num_xcc", 1);
      g.lds_kb = (int)u64(m, "lds_size_in_kb");
      g.wave_size = (int)u64(m, "wave_front_size");
      g.max_clock_mhz = (int)u64(m, "max_engine_clk_fcompute");
      g.unique_id = u64(m, "unique_id");
      g.hive_id = u64(m, "hive_id");
      g.bdf = bdf_from(u64(m, "domain"), u64(m, "location_id"));
      g.gpu_id = (uint32_t)read_int_file(nd + "/gpu_id", 0);
      for (int b : numeric_entries(nd + "/mem_banks")) {
        bool mok = false;
        auto mm = read_props(nd + "/mem_banks/" + std::to_string(b) + "/properties", &mok);
        if (mok) g.vram_bytes += u64(mm, "size_in_bytes");
      }
      g.numa_node = read_int_file(join(root, "/sys/class/drm/renderD" + std::to_string(g.render_minor) +
                                             "/device/numa_node"), -1);
    } else {
      // Unreadable node (cgroup-restricted on shared hosts): a GPU we cannot use
      // from here. Record only if a gpu_id says it is a GPU.
      int gid = read_int_file(nd + "/gpu_id", 0);
      if (gid == 0) continue;
      g.gpu_id = (uint32_t)gid;
    }
    for (const char* kind : {"io_links", "p2p_links"}) {
      for (int l : numeric_entries(nd + "/" + kind)) {
        bool lok = false;
        auto lm = read_props(nd + "/" + kind + "/" + std::to_string(l) + "/properties", &lok);
        if (!lok) continue;
        Link L;
        L.to_node = (int)u64(lm, "node_to", (uint64_t)-1);
        L.type = (int)u64(lm, "type");
        L.weight = (int)u64(lm, "weight");
        L.max_bandwidth_mbs = u64(lm, "max_bandwidth");
        bool dup = false;
        for (auto& e : g.links) dup |= (e.to_node == L.to_node && e.type == L.type);
        if (!dup) g.links.push_back(L);
      }
    }
    t.gpus.push_back(std::move(g));
  }
  // keep only links to GPU nodes; index GPUs
  std::vector<int> gpu_nodes;
  for (auto& g : t.gpus) gpu_nodes.push_back(g.node_id);
  for (size_t i = 0; i < t.gpus.size(); ++i) {
    auto& g = t.gpus[i];
    g.index = (int)i;
    g.links.erase(std::remove_if(g.links.begin(), g.links.end(),
                                 [&](const Link& L) {
                                   return std::find(gpu_nodes.begin(), gpu_nodes.end(), L.to_node) ==
                                          gpu_nodes.end();
                                 }),
                  g.links.end());
    refresh_health(root, g);
  }
  if (use_amdsmi && (root.empty() || root == "/")) t.amdsmi_used = enrich_with_amdsmi(t);
  if (!t.kfd_present) t.warnings.push_back("/dev/kfd not present: no usable AMD GPU (fake capacity path)");
  (void)render_nodes;
  return t;
}

std::vector<std::vector<int>> link_matrix(const Topology& t) {
  const size_t n = t.gpus.size();
  std::vector<std::vector<int>> m(n, std::vector<int>(n, 0));
  std::map<int, size_t> idx;
  for (size_t i = 0; i < n; ++i) idx[t.gpus[i].node_id] = i;
  for (size_t i = 0; i < n; ++i) {
    m[i][i] = -1;
    for (auto& L : t.gpus[i].links) {
      auto it = idx.find(L.to_node);
      if (it != idx.end()) m[i][it->second] = std::max(m[i][it->second], L.type);
    }
  }
  return m;
}

std::string to_json(const Topology& t) {
  std::ostringstream o;
  o << "{\"root\":\"" << json_escape(t.root) << "\",\"kfd_present\":" << (t.kfd_present ? "true" : "false")
    << ",\"topology_present\":" << (t.topology_present ? "true" : "false")
    << ",\"amdsmi_used\":" << (t.amdsmi_used ? "true" : "false") << ",\"cpu_nodes\":" << t.cpu_nodes
    << ",\"warnings\":[";
  for (size_t i = 0; i < t.warnings.size(); ++i) o << (i ? "," : "") << "\"" << json_escape(t.warnings[i]) << "\"";
  o << "],\"gpus\":[";
  for (size_t i = 0; i < t.gpus.size(); ++i) {
    const Gpu& g = t.gpus[i];
    o << (i ? "," : "") << "{\"index\":" << g.index << ",\"node_id\":" << g.node_id << ",\"gpu_id\":" << g.gpu_id
      << ",\"render_minor\":" << g.render_minor << ",\"bdf\":\"" << g.bdf << "\",\"unique_id\":\"" << g.unique_id
      << "\",\"hive_id\":\"" << g.hive_id << "\",\"gfx_target_version\":" << g.gfx_target_version
      << ",\"gfx_arch\":\"" << g.gfx_arch << "\",\"vendor_id\":" << g.vendor_id << ",\"device_id\":" << g.device_id
      << ",\"simd_count\":" << g.simd_count << ",\"cu_count\":" << g.cu_count << ",\"num_xcc\":" << g.num_xcc
      << ",\"lds_kb\":" << g.lds_kb << ",\"wave_size\":" << g.wave_size << ",\"max_clock_mhz\":" << g.max_clock_mhz
      << ",\"vram_bytes\":" << g.vram_bytes << ",\"numa_node\":" << g.numa_node << ",\"uuid\":\""
      << json_escape(g.uuid) << "\",\"properties_readable\":" << (g.properties_readable ? "true" : "false")
      << ",\"render_node_present\":" << (g.render_node_present ? "true" : "false")
      << ",\"healthy\":" << (g.healthy ? "true" : "false") << ",\"health_reason\":\""
      << json_escape(g.health_reason) << "\",\"links\":[";
    for (size_t j = 0; j < g.links.size(); ++j) {
      const Link& L = g.links[j];
      o << (j ? "," : "") << "{\"to_node\":" << L.to_node << ",\"type\":" << L.type << ",\"weight\":" << L.weight
        << ",\"max_bandwidth_mbs\":" << L.max_bandwidth_mbs << "}";
    }
    o << "]}";
  }
  o << "]}";
  return o.str();
}

}  // namespace gpuinfo
}  // namespace kgs
