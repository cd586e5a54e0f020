// pybind11 bindings of the native runtime: module `_bcg_runtime`.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime.h"

namespace py = pybind11;
using namespace bcg;

static py::tuple py_compile_token_fsm(py::array_t<int32_t, py::array::c_style | py::array::forcecast> trans,
                                      py::array_t<uint8_t, py::array::c_style | py::array::forcecast> accept,
                                      const std::vector<py::bytes>& tokens, int vocab_rows) {
  if (trans.ndim() != 2 || trans.shape(1) != 256) throw std::invalid_argument("trans must be [S,256]");
  const int S = static_cast<int>(trans.shape(0));
  if (accept.ndim() != 1 || accept.shape(0) != S) throw std::invalid_argument("accept must be [S]");
  if (S >= 32767) throw std::invalid_argument("too many FSM states for int16 tables");
  std::vector<std::string> toks;
  toks.reserve(tokens.size());
  for (auto& b : tokens) toks.emplace_back(std::string(b));
  TokenFsmTables t;
  {
    py::gil_scoped_release nogil;
    t = compile_token_fsm(trans.data(), accept.data(), S, toks, vocab_rows);
  }
  py::array_t<int16_t> next({S, vocab_rows});
  std::memcpy(next.mutable_data(), t.next.data(), t.next.size() * sizeof(int16_t));
  py::array_t<int16_t> dist(S);
  std::memcpy(dist.mutable_data(), t.dist.data(), t.dist.size() * sizeof(int16_t));
  return py::make_tuple(next, dist);
}

#ifndef BCG_SOURCE_HASH
#define BCG_SOURCE_HASH "unstamped"
#endif

PYBIND11_MODULE(_bcg_runtime, m) {
  m.doc() = "BCG MI355X engine native runtime (token FSM compiler, paged-KV block manager)";
  m.attr("source_hash") = BCG_SOURCE_HASH;  // utils/build.py: hash of csrc/runtime/*
  m.def("compile_token_fsm", &py_compile_token_fsm, py::arg("trans"), py::arg("accept"),
        py::arg("tokens"), py::arg("vocab_rows"));

  py::class_<Allocation>(m, "Allocation")
      .def_readonly("ok", &Allocation::ok)
      .def_readonly("blocks", &Allocation::blocks)
      .def_readonly("num_cached_tokens", &Allocation::num_cached_tokens);

  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int, int>(), py::arg("num_blocks"), py::arg("block_size"))
      .def("allocate", &BlockManager::allocate, py::arg("prompt"), py::arg("max_new_tokens"),
           py::arg("use_cache") = true)
      .def("commit_prompt", &BlockManager::commit_prompt)
      .def("free", &BlockManager::free)
      .def("reset_cache", &BlockManager::reset_cache)
      .def_property_readonly("num_free_blocks", &BlockManager::num_free_blocks)
      .def_property_readonly("num_blocks", &BlockManager::num_blocks)
      .def_property_readonly("block_size", &BlockManager::block_size)
      .def_property_readonly("hits", &BlockManager::hits)
      .def_property_readonly("lookups", &BlockManager::lookups)
      .def_property_readonly("evictions", &BlockManager::evictions)
      .def_property_readonly("cached_blocks", &BlockManager::cached_blocks);
}
