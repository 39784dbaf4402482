// pybind11 module kgs._native._gpuinfo: the device plugin's view of the GPUs.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "gpuinfo.h"

namespace py = pybind11;
using namespace kgs::gpuinfo;

PYBIND11_MODULE(_gpuinfo, m) {
  m.doc() = "kgs native GPU enumeration (KFD sysfs topology + amd-smi)";
  m.def(
      "discover_json",
      [](const std::string& root, bool use_amdsmi) {
        py::gil_scoped_release nogil;
        return to_json(discover(root, use_amdsmi));
      },
      py::arg("root") = "/", py::arg("use_amdsmi") = true);
  m.def("gfx_name", &gfx_name);
  m.def(
      "link_matrix",
      [](const std::string& root) { return link_matrix(discover(root, false)); }, py::arg("root") = "/");
  m.def(
      "health",
      [](const std::string& root, int node_id, int render_minor) {
        Gpu g;
        g.node_id = node_id;
        g.render_minor = render_minor;
        bool ok = refresh_health(root, g);
        return py::make_tuple(ok, g.health_reason);
      },
      py::arg("root"), py::arg("node_id"), py::arg("render_minor"));
  py::class_<HealthMonitor>(m, "HealthMonitor")
      .def(py::init<const std::string&, bool, int64_t>(), py::arg("root") = "/", py::arg("use_amdsmi") = true,
           py::arg("ecc_tolerance") = 0)
      .def_property_readonly("amdsmi_used", &HealthMonitor::amdsmi_used)
      .def(
          "check",
          [](HealthMonitor& hm, int node_id, int render_minor, const std::string& bdf) {
            HealthState st;
            {
              py::gil_scoped_release nogil;
              st = hm.check(node_id, render_minor, bdf);
            }
            py::dict d;
            d["healthy"] = st.healthy;
            d["reason"] = st.reason;
            d["amdsmi"] = st.smi;
            d["ecc_correctable"] = st.sample.ecc_correctable;
            d["ecc_uncorrectable"] = st.sample.ecc_uncorrectable;
            d["ecc_deferred"] = st.sample.ecc_deferred;
            d["xgmi_links_total"] = st.sample.links_total;
            d["xgmi_links_up"] = st.sample.links_up;
            d["xgmi_links_down"] = st.sample.links_down;
            return d;
          },
          py::arg("node_id"), py::arg("render_minor"), py::arg("bdf") = "");
}
