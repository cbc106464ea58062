// JIT specialisation of lowered programs (jit.cpp).
#pragma once
#include <string>
#include <vector>

#include "program.hpp"

namespace mg {

// HIP source of the requested kernels: mgj_search (generator + first hit), mgj_gen
// (per-candidate verdicts of generated candidates) and mgj_eval (SoA inputs).
// `specs`/`gconsts` (nullable) specialise the generator at codegen time.
enum : uint32_t { JIT_SEARCH = 1, JIT_EVAL = 2, JIT_GEN = 4, JIT_EVAL_TILED = 8 };
std::string jit_source(const Lowered& P, const std::vector<GenSpec>* specs, const std::vector<uint32_t>* gconsts,
                       uint32_t kernels);

// The first tier (jit_asm.cpp): the same kernels (JIT_SEARCH, optionally JIT_GEN) as gfx950 assembly
// with the emitter's own register allocation; assembled and linked by comgr in a few ms instead of
// ~140 ms of clang + LLVM.  MG_E_UNSUPPORTED (err says why) for programs outside the tier.
// Sources starting with kAsmMarker are assembled, not compiled, by jit_compile*.
constexpr const char* kAsmMarker = "; mythgpu-asm";
int jit_asm_source(const Lowered& P, const std::vector<GenSpec>& specs, const std::vector<uint32_t>& gconsts,
                   uint32_t kernels, std::string& out, std::string& err);

// Load the JIT compiler library now (on the calling thread): its static destructors then
// register before anything the caller registers with atexit afterwards.
void jit_compiler_preload();
// start the compile helpers and warm the first tier's by assembling `asm_src` (a tiny kernel) —
// mg_init runs it on a detached thread; MYTHGPU_JIT_WARM=0 or in-process compiles: nothing
void jit_helper_warm(const std::string& asm_src);

// compile for gfx950 -> code object bytes. MG_OK or MG_E_*; `log` gets the compiler log.  By
// default through the compiler helper process (mythgpu_jitd): a compiler abort there fails the
// compile, not the caller.  jit_compile_local: comgr (or hipRTC) in this process.
// from_disk (nullable): set when the code object came from the on-disk cache
int jit_compile(const std::string& src, std::vector<char>& code, std::string& log, bool* from_disk = nullptr);
// drop the on-disk cache entry of `src` (a code object the runtime refused to load)
void jit_disk_evict(const std::string& src);
int jit_compile_local(const std::string& src, std::vector<char>& code, std::string& log);

// the helper process: stop it (end of input; it exits), and its pid (-1 none yet, -2 died)
void jit_helper_stop();
int jit_helper_pid();

}  // namespace mg
