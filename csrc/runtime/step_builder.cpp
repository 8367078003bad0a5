// Native step-input builder for the decode rows of an engine step (the per-step host
// work that sits between two GPU steps: for 128-256 running sequences the Python/numpy
// version cost ~1-2 ms per step, exposed as GPU idle time).
//
// decode_rows(tables, starts, tokens, lengths, block_size, width, pad_to) ->
//   (ids[int32 P], positions[int32 P], slots[int32 P], ctx[int32 P], block_tables[int32 P x width])
// for P = max(len(starts), pad_to) rows (padding rows: id 0, position 0, slot -1, ctx 1,
// zero block table -- what the hipGraph decode buckets expect).  slot = table[pos / bs]
// * bs + pos % bs (the KV write target of the new token).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <stdexcept>
#include <vector>

namespace py = pybind11;

static py::tuple decode_rows(const std::vector<std::vector<int>>& tables, const std::vector<int>& starts,
                             const std::vector<int>& tokens, const std::vector<int>& lengths, int bs, int width,
                             int pad_to) {
  const size_t B = starts.size();
  if (tables.size() != B || tokens.size() != B || lengths.size() != B) throw std::invalid_argument("length mismatch");
  if (bs <= 0 || width <= 0) throw std::invalid_argument("bad block size / width");
  const size_t P = std::max<size_t>(B, pad_to > 0 ? (size_t)pad_to : 0);
  py::array_t<int> ids(P), pos(P), slots(P), ctx(P);
  py::array_t<int> bt({(py::ssize_t)P, (py::ssize_t)width});
  auto I = ids.mutable_unchecked<1>();
  auto Q = pos.mutable_unchecked<1>();
  auto S = slots.mutable_unchecked<1>();
  auto C = ctx.mutable_unchecked<1>();
  auto T = bt.mutable_unchecked<2>();
  for (size_t i = 0; i < P; ++i) {
    for (int j = 0; j < width; ++j) T(i, j) = 0;
    if (i >= B) {
      I(i) = 0;
      Q(i) = 0;
      S(i) = -1;
      C(i) = 1;
      continue;
    }
    const auto& t = tables[i];
    if ((int)t.size() > width) throw std::invalid_argument("block table wider than width");
    const int p = starts[i];
    const int blk = p / bs;
    if (blk >= (int)t.size()) throw std::invalid_argument("position beyond the block table");
    for (size_t j = 0; j < t.size(); ++j) T(i, j) = t[j];
    I(i) = tokens[i];
    Q(i) = p;
    S(i) = t[blk] * bs + p % bs;
    C(i) = lengths[i];
  }
  return py::make_tuple(ids, pos, slots, ctx, bt);
}

void register_step_builder(py::module_& m) {
  m.def("decode_rows", &decode_rows, py::arg("tables"), py::arg("starts"), py::arg("tokens"), py::arg("lengths"),
        py::arg("block_size"), py::arg("width"), py::arg("pad_to") = 0);
}
