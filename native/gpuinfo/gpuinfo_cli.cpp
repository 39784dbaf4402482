// kgs-gpuinfo: print the GPUs (and xGMI matrix) this host exposes.
//   kgs-gpuinfo [--root DIR] [--json] [--no-amdsmi]
#include <cstdio>
#include <cstring>
#include <string>

#include "gpuinfo.h"

using namespace kgs::gpuinfo;

int main(int argc, char** argv) {
  std::string root = "/";
  bool json = false, smi = true;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--root") && i + 1 < argc) root = argv[++i];
    else if (!std::strcmp(argv[i], "--json")) json = true;
    else if (!std::strcmp(argv[i], "--no-amdsmi")) smi = false;
    else {
      std::fprintf(stderr, "usage: %s [--root DIR] [--json] [--no-amdsmi]\n", argv[0]);
      return 2;
    }
  }
  Topology t = discover(root, smi);
  if (json) {
    std::printf("%s\n", to_json(t).c_str());
    return 0;
  }
  std::printf("root=%s kfd=%s gpus=%zu cpu_nodes=%d amdsmi=%s\n", t.root.c_str(), t.kfd_present ? "yes" : "no",
              t.gpus.size(), t.cpu_nodes, t.amdsmi_used ? "yes" : "no");
  for (auto& w : t.warnings) std::printf("warning: %s\n", w.c_str());
  std::printf("%-4s %-5s %-7s %-13s %-8s %-5s %-4s %-10s %-4s %s\n", "idx", "node", "render", "bdf", "arch", "CUs",
              "xcc", "vram_GiB", "numa", "health");
  for (auto& g : t.gpus)
    std::printf("%-4d %-5d %-7d %-13s %-8s %-5d %-4d %-10.1f %-4d %s\n", g.index, g.node_id, g.render_minor,
                g.bdf.c_str(), g.gfx_arch.c_str(), g.cu_count, g.num_xcc, g.vram_bytes / 1073741824.0, g.numa_node,
                g.health_reason.c_str());
  auto m = link_matrix(t);
  if (m.size() > 1) {
    std::printf("links (X = xGMI, P = PCIe, . = none):\n");
    for (size_t i = 0; i < m.size(); ++i) {
      std::printf("  %2zu ", i);
      for (size_t j = 0; j < m.size(); ++j)
        std::printf(" %c", m[i][j] < 0 ? '-' : m[i][j] == LINK_XGMI ? 'X' : m[i][j] == LINK_PCIE ? 'P' : '.');
      std::printf("\n");
    }
  }
  return 0;
}
