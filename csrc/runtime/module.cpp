// `_runtime` extension module: native runtime pieces of the serving engine.
#include <pybind11/pybind11.h>

namespace py = pybind11;

void register_block_allocator(py::module_& m);
void register_bpe(py::module_& m);
void register_step_builder(py::module_& m);

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "native runtime: paged-KV block allocator with prefix caching, byte-level BPE encoder, step-input builder";
  register_block_allocator(m);
  register_bpe(m);
  register_step_builder(m);
}
