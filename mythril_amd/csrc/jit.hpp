// JIT specialisation of lowered programs (jit.cpp).
#pragma once
#include <string>
#include <vector>

#include "program.hpp"

namespace mg {

// HIP source with two kernels: mgj_search (generator + first hit) and mgj_eval (SoA inputs).
// `specs`/`gconsts` (nullable) specialise the generator at codegen time.
std::string jit_source(const Lowered& P, const std::vector<GenSpec>* specs, const std::vector<uint32_t>* gconsts,
                       bool want_search, bool want_eval);

// hipRTC compile for gfx950 -> code object bytes. MG_OK or MG_E_*; `log` gets the compiler log.
int jit_compile(const std::string& src, std::vector<char>& code, std::string& log);

}  // namespace mg
