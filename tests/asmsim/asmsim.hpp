// A CPU simulator of the gfx950 instruction subset the first JIT tier emits
// (mythril_amd/csrc/jit_asm.cpp) and the O3 tier's compiler output uses (disassembled by
// tools/o3dis.py) — test infrastructure only, never linked into the product.
//
// It runs the emitted kernels (mgj_search, mgj_gen, mgj_eval) wave by wave on the host, 64 lanes
// per wave, four waves per 256-lane block, with a flat 64-bit memory of the buffers the engine
// would pass, so the first tier's output can be compared per candidate with the C port
// (oracle/bveval.c) on any number of programs without a GPU.  Besides the arithmetic it checks
// the rules the emitter claims to keep; any violation is an error, not a wrong verdict:
//   * a VGPR or SGPR read (or overwritten) while a load into it is still in flight (vmcnt /
//     lgkmcnt not waited for), loads returning in issue order per counter;
//   * a VALU read of an SGPR (VCC included) fewer than 2 wait states after a VALU wrote it, and a
//     VMEM read of an SGPR fewer than 5 after a VALU wrote it (s_nop N = N + 1 wait states);
//   * the constant bus: one SGPR or literal per VALU instruction (implicit VCC included), no
//     32-bit literal in a VOP3 encoding;
//   * an access outside every buffer, or outside the kernel's LDS allocation;
//   * a read of a VGPR no instruction wrote in this wave;
//   * a kernel that runs more than a step budget (a wave that never exits).
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

namespace asmsim {

struct SimError {
  std::string what;
};

enum OKind : uint8_t { O_NONE, O_V, O_S, O_IMM, O_EXEC, O_OFF };
struct Opd {
  OKind k = O_NONE;
  int r = 0;       // register number (vcc = s106)
  int n = 1;       // registers (a pair: 2)
  uint64_t imm = 0;
  bool inl = false;  // an inline constant (-16..64)
};

struct Ins {
  int op = 0;
  std::vector<Opd> a;
  int64_t offset = 0;   // offset:N
  int vmcnt = -1, lgkmcnt = -1;  // s_waitcnt
  int sdwa_src1_word1 = 0;
  int sdwa_sel[2] = {0, 0};  // SDWA source selects: 0 DWORD, 1 WORD_0, 2 WORD_1, 3..6 BYTE_0..3
  int offset0 = 0, offset1 = 0;  // ds_read2 / ds_write2 (dwords)
  int enc = 0;          // 0 VOP3-only / none, 1 _e32, 2 _e64, 3 _sdwa
  int bitop3 = -1;      // v_bitop3_b32's table
  int target = -1;      // branch target (instruction index)
  std::string text;     // the source line (diagnostics)
  int tag = -1;         // the "; vcode ..." annotation region it belongs to (MYTHGPU_JIT_ASM_ANNOTATE)
  int64_t pc = -1;      // code address (".asmsim_pc A" before it; s_getpc_b64 of compiled code)
};

struct Kernel {
  size_t entry = 0;
  uint32_t lds_bytes = 0;
};

struct Module {
  std::vector<Ins> code;
  std::map<std::string, Kernel> kernels;
  std::vector<std::string> tags;  // annotation texts, by Ins::tag
  // ".asmsim_image <file>": the code object's loaded image (vaddr 0 up), mapped at a buffer of its
  // own so that s_getpc_b64-relative reads of baked tables (the O3 tier's mg_gd) find their data
  std::vector<uint8_t> image;
};

// parse the emitter's assembly text (throws SimError on anything unknown)
Module parse(const std::string& text);

struct Buffer {
  uint64_t base = 0;
  std::vector<uint8_t> data;
};

struct Memory {
  std::vector<Buffer> bufs;
  uint64_t add(size_t bytes, const void* init = nullptr);  // returns the base address
  uint8_t* at(uint64_t addr, size_t n);
  Buffer& of(uint64_t base);
};

struct Stats {
  uint64_t insts = 0, valu = 0, salu = 0, vmem = 0, lds = 0, waves = 0;
  // extra LDS cycles from bank conflicts (the gfx950 lane groups and banks of
  // docs MI355X_MICROARCH.md §LDS; what SQ_LDS_BANK_CONFLICT counts)
  uint64_t lds_conflict = 0;
  uint64_t nop_slots = 0, branches = 0, waitcnts = 0;  // s_nop wait states, branches, s_waitcnt
  std::map<int, uint64_t> valu_by_tag;  // VALU wave-instructions per annotation region
  std::map<int, uint64_t> salu_by_tag;  // SALU instructions per annotation region
};

// run `kernel` over `nblk` 256-lane blocks; kernarg: the argument block's address
void launch(const Module& m, const std::string& kernel, Memory& mem, uint64_t kernarg, uint32_t nblk,
            Stats* stats = nullptr, uint64_t max_steps = 400000000ull);

}  // namespace asmsim
