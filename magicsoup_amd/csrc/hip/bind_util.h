// Bindings of the device core: every function is wrapped so that the kernels it records go out as one
// graph launch when it returns (launch.h BatchGuard). gdef(m, name, f, extra...) == m.def(name, f,
// extra...) with that wrapper.
#pragma once
#include <pybind11/pybind11.h>

#include <type_traits>
#include <utility>

#include "launch.h"

namespace msd {

template <class R, class... A>
auto batch_wrapped(R (*f)(A...)) {
  return [f](A... a) -> R {
    BatchGuard g;
    if constexpr (std::is_void_v<R>) {
      f(std::forward<A>(a)...);
      g.finish();
    } else {
      R r = f(std::forward<A>(a)...);
      g.finish();
      return r;
    }
  };
}

template <class F, class R, class C, class... A>
auto batch_wrapped_call(F f, R (C::*)(A...) const) {
  return [f](A... a) -> R {
    BatchGuard g;
    if constexpr (std::is_void_v<R>) {
      f(std::forward<A>(a)...);
      g.finish();
    } else {
      R r = f(std::forward<A>(a)...);
      g.finish();
      return r;
    }
  };
}

template <class F>
auto batch_wrapped(F f) {
  return batch_wrapped_call(f, &F::operator());
}

template <class F, class... Extra>
void gdef(pybind11::module_& m, const char* name, F&& f, const Extra&... extra) {
  m.def(name, batch_wrapped(std::forward<F>(f)), extra...);
}

}  // namespace msd
