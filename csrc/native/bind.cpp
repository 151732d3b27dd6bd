// pybind11 bindings of the host native runtime.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "native.h"

namespace py = pybind11;
using namespace ytk_native;

PYBIND11_MODULE(_ytk_native, m) {
  m.doc() = "ytk-learn-amd native host runtime";
  m.def("murmur3_128_aslong", [](const std::string& s, uint32_t seed) {
    return murmur3_128_aslong(s.data(), s.size(), seed);
  });
  m.def("murmur3_128_aslong_many", [](const std::vector<std::string>& names, uint32_t seed) {
    py::array_t<int64_t> out(names.size());
    auto o = out.mutable_unchecked<1>();
    for (size_t i = 0; i < names.size(); ++i)
      o(i) = murmur3_128_aslong(names[i].data(), names[i].size(), seed);
    return out;
  });
}
