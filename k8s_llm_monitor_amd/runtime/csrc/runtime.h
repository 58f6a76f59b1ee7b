// Registration hooks of the native runtime's translation units (one pybind11 module).
#pragma once
#include <pybind11/pybind11.h>

void register_step_channel(pybind11::module_& m);
