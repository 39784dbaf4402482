// pybind11 binding of the kgs.serve scheduler (module kgs._native._serve).
// Step plans come back as numpy int32/int64 arrays ready for one pinned
// host->device copy each.
#include <cstring>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "scheduler.h"

namespace py = pybind11;
using namespace kgs::serve;

template <typename T>
static py::array_t<T> arr(const std::vector<T>& v) {
  py::array_t<T> a((py::ssize_t)v.size());
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

PYBIND11_MODULE(_serve, m) {
  m.doc() = "kgs.serve native continuous-batching scheduler and paged-KV block allocator";

  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int>(), py::arg("num_pages"))
      .def("alloc", &BlockAllocator::alloc)
      .def("free", &BlockAllocator::free)
      .def_property_readonly("num_free", &BlockAllocator::num_free)
      .def_property_readonly("num_pages", &BlockAllocator::num_pages);

  py::class_<SchedulerConfig>(m, "SchedulerConfig")
      .def(py::init<>())
      .def_readwrite("num_pages", &SchedulerConfig::num_pages)
      .def_readwrite("page_size", &SchedulerConfig::page_size)
      .def_readwrite("max_batch", &SchedulerConfig::max_batch)
      .def_readwrite("max_prefill_tokens", &SchedulerConfig::max_prefill_tokens)
      .def_readwrite("max_model_len", &SchedulerConfig::max_model_len)
      .def_readwrite("pad_multiple", &SchedulerConfig::pad_multiple)
      .def_readwrite("chunk_tokens", &SchedulerConfig::chunk_tokens)
      .def_readwrite("prefix_caching", &SchedulerConfig::prefix_caching);

  py::class_<StepPlan>(m, "StepPlan")
      .def_readonly("kind", &StepPlan::kind)
      .def_readonly("max_pages", &StepPlan::max_pages)
      .def_property_readonly("seq_ids", [](const StepPlan& p) { return arr(p.seq_ids); })
      .def_property_readonly("tokens", [](const StepPlan& p) { return arr(p.tokens); })
      .def_property_readonly("positions", [](const StepPlan& p) { return arr(p.positions); })
      .def_property_readonly("slots", [](const StepPlan& p) { return arr(p.slots); })
      .def_property_readonly("seq_starts", [](const StepPlan& p) { return arr(p.seq_starts); })
      .def_property_readonly("seq_lens", [](const StepPlan& p) { return arr(p.seq_lens); })
      .def_property_readonly("padded_lens", [](const StepPlan& p) { return arr(p.padded_lens); })
      .def_property_readonly("block_tables",
                             [](const StepPlan& p) {
                               auto a = arr(p.block_tables);
                               if (p.max_pages > 0) a.resize({(py::ssize_t)p.ctx_lens.size(), (py::ssize_t)p.max_pages});
                               return a;
                             })
      .def_property_readonly("ctx_lens", [](const StepPlan& p) { return arr(p.ctx_lens); })
      .def_property_readonly("preempted", [](const StepPlan& p) { return arr(p.preempted); })
      .def_readonly("n_prefill", &StepPlan::n_prefill)
      .def_readonly("pf_max_pages", &StepPlan::pf_max_pages)
      .def_property_readonly("ctx_starts", [](const StepPlan& p) { return arr(p.ctx_starts); })
      .def_property_readonly("last_chunk", [](const StepPlan& p) { return arr(p.last_chunk); })
      .def_property_readonly("pf_block_tables", [](const StepPlan& p) {
        auto a = arr(p.pf_block_tables);
        if (p.pf_max_pages > 0) a.resize({(py::ssize_t)p.n_prefill, (py::ssize_t)p.pf_max_pages});
        return a;
      });

  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<const SchedulerConfig&>(), py::arg("config"))
      .def("add", &Scheduler::add, py::arg("id"), py::arg("prompt"), py::arg("max_new_tokens"))
      .def("abort", &Scheduler::abort)
      .def("schedule", &Scheduler::schedule)
      .def(
          "update",
          [](Scheduler& s, py::array_t<int64_t> ids, py::array_t<int32_t> toks, py::array_t<uint8_t> eos) {
            auto i = ids.unchecked<1>();
            auto t = toks.unchecked<1>();
            auto e = eos.unchecked<1>();
            std::vector<int64_t> vi(i.shape(0));
            std::vector<int32_t> vt(t.shape(0));
            std::vector<uint8_t> ve(e.shape(0));
            for (py::ssize_t k = 0; k < i.shape(0); ++k) vi[k] = i(k);
            for (py::ssize_t k = 0; k < t.shape(0); ++k) vt[k] = t(k);
            for (py::ssize_t k = 0; k < e.shape(0); ++k) ve[k] = e(k);
            return arr(s.update(vi, vt, ve));
          },
          py::arg("ids"), py::arg("tokens"), py::arg("eos"))
      .def("update_pending",
           [](Scheduler& s, py::array_t<int64_t> ids) {
             auto i = ids.unchecked<1>();
             std::vector<int64_t> vi(i.shape(0));
             for (py::ssize_t k = 0; k < i.shape(0); ++k) vi[k] = i(k);
             return arr(s.update_pending(vi));
           },
           py::arg("ids"))
      .def("fill_pending",
           [](Scheduler& s, py::array_t<int64_t> ids, py::array_t<int32_t> toks) {
             auto i = ids.unchecked<1>();
             auto t = toks.unchecked<1>();
             std::vector<int64_t> vi(i.shape(0));
             std::vector<int32_t> vt(t.shape(0));
             for (py::ssize_t k = 0; k < i.shape(0); ++k) vi[k] = i(k);
             for (py::ssize_t k = 0; k < t.shape(0); ++k) vt[k] = t(k);
             return s.fill_pending(vi, vt);
           },
           py::arg("ids"), py::arg("tokens"))
      .def_property_readonly_static("PENDING", [](py::object) { return Scheduler::kPendingToken; })
      .def("tokens",
           [](const Scheduler& s, int64_t id) {
             const Sequence* q = s.get(id);
             if (!q) throw py::key_error("unknown sequence");
             return arr(q->tokens);
           })
      .def("info",
           [](const Scheduler& s, int64_t id) {
             const Sequence* q = s.get(id);
             if (!q) throw py::key_error("unknown sequence");
             py::dict d;
             d["prompt_len"] = q->prompt_len;
             d["generated"] = q->generated;
             d["state"] = (int)q->state;
             d["cached"] = q->cached;
             d["pages"] = q->pages.size();
             d["preemptions"] = q->preemptions;
             return d;
           })
      .def("release", &Scheduler::release)
      .def_property_readonly("num_waiting", &Scheduler::num_waiting)
      .def_property_readonly("num_running", &Scheduler::num_running)
      .def_property_readonly("num_free_pages", &Scheduler::num_free_pages)
      .def_property_readonly("prefix_hit_tokens", &Scheduler::prefix_hit_tokens)
      .def_property_readonly("num_cached_pages", &Scheduler::num_cached_pages)
      .def("check_invariants", &Scheduler::check_invariants);
}
