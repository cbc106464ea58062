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

// What a code object asks of the runtime, read from its AMDHSA kernel descriptors (every `*.kd`
// symbol): the largest private (scratch) segment per lane, whether any kernel uses a dynamic stack
// (kernel_code_properties bit 11), and how many kernels it holds.  MG_OK, or MG_E_INVALID for a
// blob that is not a gfx950 ELF code object with kernel descriptors.
struct CodeObjectInfo {
  uint32_t kernels = 0;
  uint32_t max_private_bytes = 0;
  uint32_t max_group_bytes = 0;
  bool dynamic_stack = false;
  uint32_t eval_cpb = 0;  // mgj_meta_eval_cpb: candidates per workgroup of a loop-free eval kernel (0: loops)
};
int code_object_info(const void* code, size_t len, CodeObjectInfo& out, std::string& err);
// The load gate jit_compile applies to every code object, compiled or from the disk cache: a kernel
// with a dynamic stack, or with more than MYTHGPU_JIT_PRIVATE_CAP bytes (default 16 KiB) of private
// segment per lane, or more than 160 KiB of LDS, is refused with MG_E_UNSUPPORTED before anything
// loads it (round 5's -O0 read-back kernel kept 52 KB per lane on a dynamic stack and faulted:
// profiles/r05n_gpu_pytest_O0_fault.log).  jit_refused_total counts refusals for mg_stats.
int jit_check_code_object(const std::vector<char>& code, std::string& why);
// the gate's verdict on descriptors already read (MG_OK or MG_E_UNSUPPORTED with `why`), uncounted
int code_object_gate(const CodeObjectInfo& ci, std::string& why);
uint64_t jit_refused_total();

// the helper process: stop it (end of input; it exits), and its pid (-1 none yet, -2 died)
void jit_helper_stop();
int jit_helper_pid();

}  // namespace mg
