// Host-only fuzz driver for the untrusted-input parsers of libmythgpu: the program
// parser/lowerer (lower_program), the generator parser (parse_gen), the specialiser
// (specialize_program) and the JIT source emitter (jit_source).  Built with
// -fsanitize=address,undefined by tests/test_fuzz_host.py (g++, no GPU), which feeds
// it hypothesis-mutated blobs; any sanitizer report aborts the process.
//
// stdin: a stream of records
//   u32 prog_len | prog bytes | u32 gen_words (0xFFFFFFFF = no generator) | gen words
// stdout: "records=N lowered=A gen_ok=B specialised=C"
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../mythril_amd/csrc/jit.hpp"
#include "../../mythril_amd/csrc/program.hpp"

using namespace mg;

static bool rd(FILE* f, void* p, size_t n) { return n == 0 || fread(p, 1, n, f) == n; }

int main() {
  FILE* in = stdin;
  uint64_t records = 0, lowered = 0, gen_ok = 0, specialised = 0;
  for (;;) {
    uint32_t plen;
    if (!rd(in, &plen, 4)) break;
    std::vector<uint8_t> prog(plen);
    if (!rd(in, prog.data(), plen)) return 3;
    uint32_t gw;
    if (!rd(in, &gw, 4)) return 3;
    std::vector<uint32_t> gen;
    const bool has_gen = gw != 0xFFFFFFFFu;
    if (has_gen) {
      gen.resize(gw);
      if (!rd(in, gen.data(), 4ull * gw)) return 3;
    }
    records++;
    Lowered low;
    std::string err;
    // the exact byte count, in a buffer of exactly that size: ASan sees any over-read
    uint8_t* exact = new uint8_t[plen ? plen : 1];
    for (uint32_t i = 0; i < plen; i++) exact[i] = prog[i];
    const int rc = lower_program(exact, plen, low, err);
    delete[] exact;
    if (rc != MG_OK) continue;
    lowered++;
    Lowered sp;
    if (specialize_program(low, nullptr, nullptr, sp, err) == MG_OK) (void)jit_source(sp, nullptr, nullptr, JIT_EVAL);
    if (!has_gen) continue;
    std::vector<GenSpec> specs;
    std::vector<uint32_t> consts;
    uint32_t* gexact = new uint32_t[gw ? gw : 1];
    for (uint32_t i = 0; i < gw; i++) gexact[i] = gen[i];
    const int grc = parse_gen(low, gexact, gw, specs, consts, err);
    delete[] gexact;
    if (grc != MG_OK) continue;
    gen_ok++;
    for (int keep = 0; keep < 2; keep++) {
      Lowered g;
      if (specialize_program(low, &specs, &consts, g, err, keep != 0) != MG_OK) continue;
      specialised++;
      // the engine compiles the search variant (keep_watch = false) as mgj_search + mgj_gen
      if (!keep) (void)jit_source(g, &specs, &consts, JIT_SEARCH | JIT_GEN);
    }
  }
  printf("records=%llu lowered=%llu gen_ok=%llu specialised=%llu\n", (unsigned long long)records,
         (unsigned long long)lowered, (unsigned long long)gen_ok, (unsigned long long)specialised);
  return 0;
}
