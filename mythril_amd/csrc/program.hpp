// Program v1 parser + lowering to the device instruction stream.
//
// Host-only C++ (no HIP); compiled into libmythgpu.so and also testable on a
// CPU-only machine through mg_program_check().
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/mythgpu.h"

namespace mg {

// Device instruction ops (after lowering). Arrays and UF applications are gone:
// SELECT-over-store-chains become EQ/ITE chains over a canonicalising LOOKUP.
enum KOp : uint32_t {
  K_CONST = 0,   // dst <- consts[p0 ..]
  K_COORD,       // dst <- coordinate p0 (eval: SoA row p1; search: generator)
  K_ADD, K_SUB, K_MUL, K_UDIV, K_UREM, K_SDIV, K_SREM, K_SMOD,
  K_AND, K_OR, K_XOR, K_NOT, K_NEG,
  K_SHL, K_LSHR, K_ASHR,
  K_CONCAT,      // dst <- a:b ; p1 = width(b)
  K_EXTRACT,     // dst <- a[lo +: wd] ; p0 = lo, p1 = width(a)
  K_ZEXT,        // p1 = width(a)
  K_SEXT,        // p1 = width(a)
  K_ITE,         // dst <- a ? b : c
  K_EQ, K_ULT, K_ULE, K_SLT, K_SLE,   // p1 = operand width
  K_UMUL_NOOVF,  // p1 = operand width
  K_EXP,
  K_LOOKUP,      // dst <- first prior (key==a) value, else slot p0 ; b = key width, c = n_prior, p1 = aux offset
  K_KECCAK,      // dst <- keccak256(bytes of a) ; p0 = byte length, a = MG_NONE for empty input
  K_ASSERT,      // verdict &= a ; may early-exit the wave
  K_WATCH,       // watch rows [p0 .. p0+L) <- a  (eval only)
  K_COPY,        // dst <- a
  // interpreter only (slot code, never in vcode): verdict &= (a <cmp> b) ^ neg, where
  // p0 = cmp op (K_EQ/K_ULT/K_ULE/K_SLT/K_SLE) | neg << 8, p1 = operand width; the fusion of a
  // compare whose one use is an ASSERT (through at most one NOT) — one dispatch instead of 2-3
  K_ASSERT_CMP,
  K_COUNT
};

struct Instr {
  uint32_t op, wd, dst, a, b, c, p0, p1;
};
static_assert(sizeof(Instr) == 32, "Instr must be 8 words");

struct GenSpec {
  uint32_t kind, p[7];
};

struct Lowered {
  std::vector<Instr> code;
  std::vector<uint32_t> consts;
  std::vector<uint32_t> aux;          // LOOKUP prior lists: pairs (key slot, value slot)
  uint32_t value_words = 0;
  uint32_t n_hoisted = 0;             // code[0, n_hoisted): K_CONSTs the interpreter runs once per thread
  uint32_t n_nodes = 0, n_roots = 0, n_coords = 0, n_watch = 0;
  std::vector<uint32_t> coord_width;
  std::vector<uint32_t> coord_row;    // SoA row offset of each coordinate
  std::vector<uint32_t> coord_kind;
  std::vector<uint32_t> coord_lazy;   // node providing a lazy default (MG_NONE if none)
  uint32_t coord_words = 0;
  std::vector<uint32_t> watch_row;
  uint32_t watch_words = 0;
  uint64_t limb_ops = 0;              // fixed cost table, per candidate
  uint32_t max_width = 0;
  // SSA form of the same code (operands are value ids, not slots) for the JIT
  std::vector<Instr> vcode;           // LOOKUP: p0 = default vid, p1 = offset into vaux
  std::vector<uint32_t> vaux;         // LOOKUP prior lists: pairs (key vid, value vid)
  std::vector<uint32_t> vwidth;       // width of each value id
  // the interpreter's SSA program where it differs from vcode (narrowed literal-tail keys),
  // before fusion and slots; empty: the same as vcode
  std::vector<Instr> ivcode;
  std::vector<uint32_t> ivaux;
};

// Parse + validate + lower. Returns MG_OK or an MG_E_* code with `err` set.
int lower_program(const uint8_t* blob, size_t len, Lowered& out, std::string& err);

// Fixed algorithmic cost table (32-bit limb ops), SURVEY.md §8(d).
uint64_t op_cost(uint32_t node_op, uint32_t width, uint32_t operand_width);


// Specialise a lowered program for a generator (specs/gconsts) or, with specs == nullptr,
// for explicit coordinates: range-decided compares folded, aliases renamed, dead code
// removed, slots re-allocated.  Same verdicts for every candidate the generator draws.
// keep_watch = false drops the K_WATCH instructions (and what only they used): the
// search variant; per-candidate verdicts with the model (mg_eval_generated) run the
// keep_watch variant.  keep_asserts = false also drops the asserts: the model read-back of a
// candidate already known to satisfy them evaluates only what the watch list needs.
int specialize_program(const Lowered& in, const std::vector<GenSpec>* specs, const std::vector<uint32_t>* gconsts,
                       Lowered& out, std::string& err, bool keep_watch = true, bool keep_asserts = true);

// Validate a generator blob against a lowered program; fills specs/consts.
int parse_gen(const Lowered& prog, const uint32_t* blob, size_t n_words, std::vector<GenSpec>& specs,
              std::vector<uint32_t>& consts, std::string& err);

}  // namespace mg
