// Host-runtime sanitizer driver (SURVEY.md §5 "race detection / sanitizers"):
// an executable built with -fsanitize=address,undefined that embeds CPython,
// registers the `_rt` bindings (block manager, detokenizer, JSON token FSM) as
// the built-in module `_rt_san`, and runs a Python entry point -- normally
// pytest over the runtime tests with FT_RT_MODULE=_rt_san, so every C++ call
// the engine makes is checked for out-of-bounds / use-after-free / UB.
// Built and run by tests/unit/test_sanitizers.py (plain g++, no GPU).
#include <pybind11/embed.h>

#include <cstdio>
#include <string>
#include <vector>

namespace py = pybind11;

void ftrt_register(py::module_& m);

PYBIND11_EMBEDDED_MODULE(_rt_san, m) { ftrt_register(m); }

int main(int argc, char** argv) {
  py::scoped_interpreter guard{};
  try {
    py::module_ sys = py::module_::import("sys");
    py::list args;
    for (int i = 1; i < argc; ++i) args.append(py::str(argv[i]));
    sys.attr("argv") = args;
    // argv[1:] = pytest arguments
    py::module_ pytest = py::module_::import("pytest");
    py::object rc = pytest.attr("main")(args);
    const int code = rc.cast<int>();
    std::fflush(stdout);
    return code;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "rt_sanitize: %s\n", e.what());
    return 3;
  }
}
