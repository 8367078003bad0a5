// `_runtime` extension module: native runtime pieces of the serving engine.
#include <pybind11/pybind11.h>

namespace py = pybind11;

void register_block_allocator(py::module_& m);
void register_bpe(py::module_& m);
void register_step_builder(py::module_& m);

#ifndef LK_SOURCE_STAMP
#define LK_SOURCE_STAMP "LKSTAMP:unstamped"
#endif
// build provenance (native/runtime.py passes the content hash of csrc/runtime + flags)
extern "C" __attribute__((used, visibility("default"))) const char lk_runtime_stamp[] = LK_SOURCE_STAMP;

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "native runtime: paged-KV block allocator with prefix caching, byte-level BPE encoder, step-input builder";
  m.def("source_stamp", [] { return std::string(lk_runtime_stamp + 8); });
  register_block_allocator(m);
  register_bpe(m);
  register_step_builder(m);
}
