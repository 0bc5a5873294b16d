// pybind11 entry point of the OpenMP host module magicsoup_amd._host.
#include "host_common.h"

namespace ms_host {
void bind_genetics(py::module_& m);
void bind_mutations(py::module_& m);
void bind_kinetics(py::module_& m);
void bind_world(py::module_& m);
void bind_io(py::module_& m);
}  // namespace ms_host

PYBIND11_MODULE(_host, m) {
  m.doc() = "magicsoup_amd host (CPU/OpenMP) native core";
  ms_host::bind_genetics(m);
  ms_host::bind_mutations(m);
  ms_host::bind_kinetics(m);
  ms_host::bind_world(m);
  ms_host::bind_io(m);
}
