// kgs gpuinfo core: KFD sysfs topology parser + optional amd-smi enrichment.
// See gpuinfo.h for the model. C++17, no ROCm link-time dependency: amd-smi is
// dlopen'ed so the device-plugin image does not need ROCm installed.
#include "gpuinfo.h"

#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>


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

// ---- amd-smi (optional, smi.cpp) -------------------------------------------
// UUID, health sample and the GPU-to-GPU link view, cross-checked against the
// KFD io_links: both must agree on which pairs are xGMI peers.
bool enrich_with_amdsmi(Topology& t) {
  auto s = SmiSession::open();
  if (!s) return false;
  t.amdsmi_library = s->library();
  std::vector<const SmiGpu*> sg(t.gpus.size(), nullptr);
  bool any = false;
  for (size_t i = 0; i < t.gpus.size(); ++i) {
    Gpu& g = t.gpus[i];
    const SmiGpu* x = s->by_minor(g.render_minor);
    if (!x) x = s->by_bdf(g.bdf);
    sg[i] = x;
    if (!x) continue;
    any = true;
    if (!x->uuid.empty()) g.uuid = x->uuid;
    SmiHealth h;
    if (s->health(*x, h)) {
      g.ecc_correctable = h.ecc_correctable;
      g.ecc_uncorrectable = h.ecc_uncorrectable;
      g.ecc_deferred = h.ecc_deferred;
      g.xgmi_links_total = h.links_total;
      g.xgmi_links_up = h.links_up;
      g.xgmi_links_down = h.links_down;
    }
  }
  std::map<int, size_t> idx;
  for (size_t i = 0; i < t.gpus.size(); ++i) idx[t.gpus[i].node_id] = i;
  bool checked = false, agrees = true;
  for (size_t i = 0; i < t.gpus.size(); ++i) {
    if (!sg[i]) continue;
    for (size_t j = 0; j < t.gpus.size(); ++j) {
      if (j == i || !sg[j]) continue;
      SmiLink L = s->link(*sg[i], *sg[j]);
      if (!L.ok) continue;
      SmiPeer p;
      p.to_index = (int)j;
      p.type = L.type;
      p.hops = L.hops;
      p.weight = L.weight;
      p.p2p = L.p2p;
      t.gpus[i].smi_links.push_back(p);
      int kfd = 0;
      for (auto& kl : t.gpus[i].links) {
        auto it = idx.find(kl.to_node);
        if (it != idx.end() && it->second == j) kfd = std::max(kfd, kl.type);
      }
      checked = true;
      if ((L.type == 11) != (kfd == 11)) {
        agrees = false;
        t.warnings.push_back("amd-smi and KFD disagree on GPU " + std::to_string(i) + " -> " + std::to_string(j) +
                             ": amd-smi link type " + std::to_string(L.type) + ", KFD io_link type " +
                             std::to_string(kfd));
      }
    }
  }
  t.smi_topology_checked = checked;
  t.smi_topology_agrees = checked && agrees;
  return any;
}

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

bool amdsmi_allowed(const std::string& root, bool use_amdsmi) {
  if (!use_amdsmi) return false;
  if (root.empty() || root == "/") return true;
  const char* stub = std::getenv("KGS_AMDSMI_LIB");
  return stub && *stub;
}

HealthMonitor::HealthMonitor(const std::string& root, bool use_amdsmi, int64_t ecc_tolerance)
    : root_(root.empty() ? "/" : root), tol_(ecc_tolerance < 0 ? 0 : ecc_tolerance) {
  if (amdsmi_allowed(root_, use_amdsmi)) smi_ = SmiSession::open();
}

HealthState HealthMonitor::check(int node_id, int render_minor, const std::string& bdf) {
  HealthState st;
  Gpu g;
  g.node_id = node_id;
  g.render_minor = render_minor;
  st.healthy = refresh_health(root_, g);
  st.reason = g.health_reason;
  if (!smi_) return st;
  const SmiGpu* x = smi_->by_minor(render_minor);
  if (!x) x = smi_->by_bdf(bdf);
  if (!x || !smi_->health(*x, st.sample)) return st;
  st.smi = true;
  auto it = base_.find(render_minor);
  if (it == base_.end()) {
    Base b;
    b.uncorr = st.sample.ecc_uncorrectable;
    b.links = st.sample.link_state;
    it = base_.emplace(render_minor, b).first;
  }
  Base& b = it->second;
  const int64_t u = st.sample.ecc_uncorrectable;
  if (st.sample.ecc_ok && b.uncorr >= 0 && u >= 0 && u < b.uncorr) b.uncorr = u;  // counters reset: re-baseline
  if (b.uncorr < 0 && st.sample.ecc_ok) b.uncorr = u;
  if (!st.healthy) return st;  // the sysfs verdict (device gone) stands
  if (st.sample.ecc_ok && b.uncorr >= 0 && u - b.uncorr > tol_) {
    st.healthy = false;
    st.reason = "uncorrectable ECC errors rose from " + std::to_string(b.uncorr) + " to " + std::to_string(u);
    return st;
  }
  if (st.sample.links_ok) {
    for (size_t i = 0; i < b.links.size() && i < st.sample.link_state.size(); ++i) {
      if (b.links[i] == 1 && st.sample.link_state[i] == 0) {
        st.healthy = false;
        st.reason = "xGMI link " + std::to_string(i) + " down (up at start)";
        return st;
      }
    }
  }
  st.reason = "ok (amd-smi: ECC uncorrectable " + std::to_string(u) + ", xGMI links up " +
              std::to_string(st.sample.links_up) + "/" + std::to_string(st.sample.links_total) + ")";
  return st;
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
  if (amdsmi_allowed(root, use_amdsmi)) t.amdsmi_used = enrich_with_amdsmi(t);
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
    << ",\"amdsmi_used\":" << (t.amdsmi_used ? "true" : "false") << ",\"amdsmi_library\":\""
    << json_escape(t.amdsmi_library) << "\",\"smi_topology_checked\":" << (t.smi_topology_checked ? "true" : "false")
    << ",\"smi_topology_agrees\":" << (t.smi_topology_agrees ? "true" : "false") << ",\"cpu_nodes\":" << t.cpu_nodes
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
      << json_escape(g.health_reason) << "\",\"ecc_correctable\":" << g.ecc_correctable
      << ",\"ecc_uncorrectable\":" << g.ecc_uncorrectable << ",\"ecc_deferred\":" << g.ecc_deferred
      << ",\"xgmi_links_total\":" << g.xgmi_links_total << ",\"xgmi_links_up\":" << g.xgmi_links_up
      << ",\"xgmi_links_down\":" << g.xgmi_links_down << ",\"smi_links\":[";
    for (size_t j = 0; j < g.smi_links.size(); ++j) {
      const SmiPeer& p = g.smi_links[j];
      o << (j ? "," : "") << "{\"to_index\":" << p.to_index << ",\"type\":" << p.type << ",\"hops\":" << p.hops
        << ",\"weight\":" << p.weight << ",\"p2p\":" << p.p2p << "}";
    }
    o << "],\"links\":[";
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
