// pybind11 module `_rt`: the host-side engine runtime (no torch / HIP deps).
#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include "block_manager.h"
#include "detok.h"

namespace py = pybind11;
using namespace ftrt;

void register_json_fsm(py::module_& m);

// The bindings are a plain function so csrc/tools/rt_sanitize.cpp can register the
// same module inside an ASan/UBSan-instrumented executable that embeds Python.
void ftrt_register(py::module_& m) {
  m.doc() = "FastTalk native engine runtime (block manager, detokenizer, token FSM)";

  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, int, bool>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("enable_prefix_caching") = true)
      .def_property_readonly("num_blocks", &BlockManager::num_blocks)
      .def_property_readonly("block_size", &BlockManager::block_size)
      .def("num_free", &BlockManager::num_free)
      .def("num_free_uncached", &BlockManager::num_free_uncached)
      .def("num_cached", &BlockManager::num_cached)
      .def("can_allocate", &BlockManager::can_allocate)
      .def("match_prefix",
           [](BlockManager& bm, py::array_t<int32_t, py::array::c_style | py::array::forcecast> t,
              int max_blocks) {
             return bm.match_prefix(t.data(), (int64_t)t.size(), max_blocks);
           })
      .def("allocate", &BlockManager::allocate)
      .def("incref", &BlockManager::incref)
      .def("free", &BlockManager::free)
      .def("commit",
           [](BlockManager& bm, const std::vector<int>& blocks,
              py::array_t<int32_t, py::array::c_style | py::array::forcecast> t, int64_t n_tokens,
              int first_block) {
             if (n_tokens > (int64_t)t.size()) throw std::out_of_range("n_tokens");
             bm.commit(blocks.data(), (int)blocks.size(), t.data(), n_tokens, first_block);
           })
      .def("reset_prefix_cache", &BlockManager::reset_prefix_cache)
      .def("refcount", &BlockManager::refcount)
      .def_property_readonly("hits", &BlockManager::hits)
      .def_property_readonly("queries", &BlockManager::queries);

  py::class_<Detokenizer>(m, "Detokenizer")
      .def(py::init([](const std::vector<py::bytes>& ids) {
        std::vector<std::string> v;
        v.reserve(ids.size());
        for (auto& b : ids) v.emplace_back(b);
        return new Detokenizer(std::move(v));
      }))
      .def("new_stream", &Detokenizer::new_stream)
      .def("release", &Detokenizer::release)
      .def("push", [](Detokenizer& d, int sid, int32_t tok) {
        std::string s = d.push(sid, tok);
        return py::str(s);
      })
      .def("push_many", [](Detokenizer& d, const std::vector<int>& sids,
                           const std::vector<int32_t>& toks) {
        auto v = d.push_many(sids, toks);
        py::list out(v.size());
        for (size_t i = 0; i < v.size(); ++i) out[i] = py::str(v[i]);
        return out;
      })
      .def("flush", [](Detokenizer& d, int sid) { return py::str(d.flush(sid)); })
      .def("decode", [](const Detokenizer& d, const std::vector<int32_t>& t) {
        return py::str(d.decode(t));
      })
      .def_property_readonly("vocab_size", &Detokenizer::vocab_size);

  register_json_fsm(m);
}

#ifndef FTRT_EMBEDDED
PYBIND11_MODULE(_rt, m) { ftrt_register(m); }
#endif
