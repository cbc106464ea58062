// Differential driver of the first JIT tier on the CPU (test infrastructure): every record is a
// program (+ generator) as the engine receives it; the driver emits the first tier's kernels
// exactly as mg_jit_compile_ex does (lower -> parse_gen -> specialise -> jit_asm_source), runs
// them on the instruction simulator (asmsim.cpp) and compares with the C port (oracle/bveval.c,
// the checker) on the same candidates:
//   kind 0: mgj_gen verdicts of [start, start + count) per candidate, and mgj_search's first hit
//           and hit count (plus the early-exit first hit, and the hit lowered into a peer's word);
//   kind 1/2: mgj_eval (row-major / tiled SoA) verdicts on random coordinate rows (masked to each
//           coordinate's width), count candidates.
// Built by tests/test_asm_sim.py with g++ (optionally -fsanitize=address,undefined).
//
// stdin records: u32 kind | u32 prog_len | prog | u32 gen_words (0xFFFFFFFF none) | gen words |
//                u64 seed | u64 start | u32 count | u32 flags (bit 0: also assemble with comgr)
// stdout: one line per record that is not "ok", then a summary line
//   "records=N ok=A outside=B mismatch=C simerror=D asmerror=E valu=V"
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <chrono>
#include <fstream>
#include <sstream>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../mythril_amd/csrc/jit.hpp"
#include "../../mythril_amd/csrc/program.hpp"
#include "asmsim.hpp"

extern "C" {
int bv_search(const uint32_t* prog, size_t prog_words, const uint32_t* gen, size_t gen_words, uint64_t seed,
              uint64_t start, uint64_t count, int threads, uint64_t* first_hit, uint64_t* n_hits, uint8_t* verdicts);
int bv_eval(const uint32_t* prog, size_t prog_words, const uint32_t* soa, uint64_t n, uint8_t* verdicts);
int bv_eval_watch(const uint32_t* prog, size_t prog_words, const uint32_t* soa, uint64_t n, uint8_t* verdicts,
                  uint32_t* watch_out);
}

using namespace mg;

namespace {

bool rd(FILE* f, void* p, size_t n) { return n == 0 || fread(p, 1, n, f) == n; }

uint64_t fmix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDull;
  x ^= x >> 33;
  x *= 0xC4CEB9FE1A85EC53ull;
  x ^= x >> 33;
  return x;
}

uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

double g_t[4];  // seconds: emission, parse, simulation, C port
struct Tm {
  int k;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  explicit Tm(int k_) : k(k_) {}
  ~Tm() { g_t[k] += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); }
};

// ASMSIM_EMIT_ONLY=1: lower, specialise and emit only (the sanitizer pass over the emitter: the
// simulator and the C port run in a separate unsanitized build, where they are several times faster)
bool emit_only() {
  static const bool on = getenv("ASMSIM_EMIT_ONLY") != nullptr;
  return on;
}

struct Counts {
  uint64_t records = 0, ok = 0, outside = 0, mismatch = 0, simerror = 0, asmerror = 0, valu = 0, cand = 0;
};

constexpr uint32_t kHitU64 = 272 + 16;  // hit buffer (kHitWords) + the peer line (engine.hip kPeerWord)

void put64(std::vector<uint8_t>& ka, size_t off, uint64_t v) { memcpy(ka.data() + off, &v, 8); }
void put32(std::vector<uint8_t>& ka, size_t off, uint32_t v) { memcpy(ka.data() + off, &v, 4); }

// the simulator's grid: at most two 256-lane blocks, so every wave loops over several groups
uint32_t grid(uint64_t lanes) {
  const uint64_t want = (lanes + 255) / 256;
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, 2));
}

std::string check_search(uint64_t rec, const std::vector<uint8_t>& prog, const std::vector<uint32_t>& gen,
                         uint64_t seed, uint64_t start, uint32_t count, bool assemble, Counts& C) {
  Lowered low, sp;
  std::string err;
  if (lower_program(prog.data(), prog.size(), low, err)) return "lower: " + err;
  std::vector<GenSpec> specs;
  std::vector<uint32_t> consts;
  if (parse_gen(low, gen.data(), gen.size(), specs, consts, err)) return "parse_gen: " + err;
  if (specialize_program(low, &specs, &consts, sp, err, /*keep_watch=*/false)) return "specialise: " + err;
  std::string src;
  int rc;
  // ASMSIM_SEARCH_SOURCE=<file>: run this kernel text instead of the first tier's (the O3 tier's
  // code object through tools/o3dis.py: its instruction counts, LDS bank conflicts and verdicts)
  const char* ext = getenv("ASMSIM_SEARCH_SOURCE");
  if (ext) {
    std::ifstream f(ext, std::ios::binary);
    if (!f) return std::string("cannot read ") + ext;
    std::stringstream ss;
    ss << f.rdbuf();
    src = ss.str();
    rc = 0;
  } else {
    Tm tm(0);
    rc = jit_asm_source(sp, specs, consts, JIT_SEARCH | JIT_GEN, src, err);
  }
  if (rc == MG_E_UNSUPPORTED) {
    C.outside++;
    if (getenv("ASMSIM_WHY")) fprintf(stderr, "outside the tier: %s\n", err.c_str());
    return "";
  }
  if (rc) return "jit_asm_source: " + err;
  if (emit_only()) {
    C.cand += count;
    return "";
  }
  if (assemble) {
#ifdef ASMSIM_ASSEMBLER
    std::vector<char> code;
    std::string log;
    if (jit_compile_local(src, code, log)) {
      C.asmerror++;
      return "assembler: " + log.substr(0, 2000);
    }
#else
    return "built without the assembler (ASMSIM_ASSEMBLER)";
#endif
  }
  // the checker: the C port on the unspecialised program
  std::vector<uint8_t> want(count);
  uint64_t cf = 0, ch = 0;
  Tm tmc(3);
  if (bv_search((const uint32_t*)prog.data(), prog.size() / 4, gen.data(), gen.size(), seed, start, count, 1, &cf, &ch,
                want.data()))
    return "C port failed";
  g_t[3] += std::chrono::duration<double>(std::chrono::steady_clock::now() - tmc.t0).count();
  tmc.t0 = std::chrono::steady_clock::now();
  tmc.k = 2;
  asmsim::Stats st;
  try {
    asmsim::Module m;
    {
      Tm tp(1);
      m = asmsim::parse(src);
    }
    const uint64_t sk = fmix64(seed ^ 0x6A09E667F3BCC908ull), sg = fmix64(seed ^ 0xBB67AE8584CAA73Bull);
    const uint64_t lanes = (start + count) - (start & ~63ull);
    const uint32_t nblk = grid(lanes);
    // mgj_gen: verdict bytes
    if (m.kernels.count("mgj_gen") && !getenv("ASMSIM_NO_GEN")) {  // ASMSIM_NO_GEN: counts of diagnostic builds
      asmsim::Memory mem;
      const uint64_t g = mem.add(std::max<size_t>(4, consts.size() * 4), consts.data());
      const uint64_t ver = mem.add(count);
      std::vector<uint8_t> ka(64, 0);
      put64(ka, 0, g);
      put64(ka, 8, start);
      put64(ka, 16, count);
      put64(ka, 24, sk);
      put64(ka, 32, sg);
      put64(ka, 40, ver);
      put32(ka, 48, nblk);
      const uint64_t kb = mem.add(ka.size(), ka.data());
      asmsim::launch(m, "mgj_gen", mem, kb, nblk, &st);
      const uint8_t* got = mem.of(ver).data.data();
      for (uint32_t i = 0; i < count; i++)
        if (got[i] != want[i]) {
          C.mismatch++;
          char b[200];
          snprintf(b, sizeof b, "mgj_gen verdict at index %llu: asm %u, C port %u (seed %llu)",
                   (unsigned long long)(start + i), got[i], want[i], (unsigned long long)seed);
          return b;
        }
    }
    // mgj_search, full sweep and early exit; the early-exit launch also lowers a peer's hit word
    for (int early = 0; early < 2; early++) {
      asmsim::Memory mem;
      const uint64_t g = mem.add(std::max<size_t>(4, consts.size() * 4), consts.data());
      std::vector<uint64_t> hb(kHitU64, 0), peer(kHitU64, 0);
      hb[0] = ~0ull;
      peer[0] = ~0ull;
      const uint64_t pb = mem.add(peer.size() * 8, peer.data());
      if (early) {
        hb[272] = 1;   // one device above this one
        hb[273] = pb;  // its hit word
      }
      const uint64_t h = mem.add(hb.size() * 8, hb.data());
      std::vector<uint8_t> ka(64, 0);
      put64(ka, 0, g);
      put64(ka, 8, start);
      put64(ka, 16, count);
      put64(ka, 24, sk);
      put64(ka, 32, sg);
      put64(ka, 40, h);
      // the early-exit pass reads the hit word with agent scope on even records and with system scope
      // (MG_SEARCH_SYSTEM_SCOPE, a device mask spanning GPUs) on odd ones
      put32(ka, 48, early ? ((rec & 1) ? 3u : 1u) : 0u);
      put32(ka, 52, nblk);
      const uint64_t kb = mem.add(ka.size(), ka.data());
      asmsim::Stats sst;
      asmsim::launch(m, "mgj_search", mem, kb, nblk, early ? nullptr : &sst);
      if (!early) {
        st.valu += sst.valu;
        st.salu += sst.salu;
        // ASMSIM_COUNT=1: the full-evaluation search launch's instructions per candidate (lane-
        // instructions, as SQ_INSTS_VALU x 64 / candidates)
        if (getenv("ASMSIM_COUNT")) {
          printf("count record %llu: valu %.1f salu %.1f lds %.2f vmem %.2f lds_conflict %.2f nop %.1f branch %.1f "
                 "waitcnt %.1f per candidate\n",
                 (unsigned long long)rec, 64.0 * sst.valu / count, 64.0 * sst.salu / count, 64.0 * sst.lds / count,
                 64.0 * sst.vmem / count, 64.0 * sst.lds_conflict / count, 64.0 * sst.nop_slots / count,
                 64.0 * sst.branches / count, 64.0 * sst.waitcnts / count);
          std::map<int, std::pair<uint64_t, uint64_t>> by;  // MYTHGPU_JIT_ASM_ANNOTATE=1: per program instruction
          for (const auto& kv : sst.valu_by_tag) by[kv.first].first = kv.second;
          for (const auto& kv : sst.salu_by_tag) by[kv.first].second = kv.second;
          for (const auto& kv : by)
            printf("count tag %s: %.2f salu %.2f\n", m.tags[kv.first].c_str(), 64.0 * kv.second.first / count,
                   64.0 * kv.second.second / count);
        }
      }
      uint64_t r[kHitU64];
      memcpy(r, mem.of(h).data.data(), sizeof r);
      uint64_t hits = r[1];
      for (uint32_t q = 1; q <= 16; q++) hits += r[16 * q];
      const uint64_t first = r[0];
      const uint64_t want_first = ch ? cf : ~0ull;
      if (first != want_first || (!early && hits != ch)) {
        C.mismatch++;
        char b[240];
        snprintf(b, sizeof b, "mgj_search%s: first %llx hits %llu, C port first %llx hits %llu",
                 early ? " (early exit)" : "", (unsigned long long)first, (unsigned long long)hits,
                 (unsigned long long)want_first, (unsigned long long)ch);
        return b;
      }
      if (early) {
        uint64_t pw;
        memcpy(&pw, mem.of(pb).data.data(), 8);
        if (pw != want_first) {
          C.mismatch++;
          return "mgj_search: the peer's hit word was not lowered to the first hit";
        }
      }
    }
  } catch (const asmsim::SimError& e) {
    C.simerror++;
    return "simulator: " + e.what;
  }
  C.valu += st.valu;
  C.cand += count;
  return "";
}

std::string check_eval(const std::vector<uint8_t>& prog, uint64_t seed, uint32_t n, bool tiled, bool assemble,
                       Counts& C) {
  Lowered low, sp;
  std::string err;
  if (lower_program(prog.data(), prog.size(), low, err)) return "lower: " + err;
  if (specialize_program(low, nullptr, nullptr, sp, err)) return "specialise: " + err;
  std::string src;
  int rc = jit_asm_source(sp, {}, {}, JIT_EVAL | (tiled ? JIT_EVAL_TILED : 0u), src, err);
  if (const char* f = getenv("ASMSIM_DUMP")) {  // debugging: the emitted text
    if (FILE* fp = fopen(f, "wb")) {
      fwrite(src.data(), 1, src.size(), fp);
      fclose(fp);
    }
  }
  if (const char* f = getenv("ASMSIM_SOURCE")) {  // debugging: simulate this text instead
    FILE* fp = fopen(f, "rb");
    if (fp) {
      src.clear();
      char buf[4096];
      size_t n;
      while ((n = fread(buf, 1, sizeof buf, fp)) > 0) src.append(buf, n);
      fclose(fp);
      rc = MG_OK;
    }
  }
  if (rc == MG_E_UNSUPPORTED) {
    C.outside++;
    if (getenv("ASMSIM_WHY")) fprintf(stderr, "outside the tier: %s\n", err.c_str());
    return "";
  }
  if (rc) return "jit_asm_source: " + err;
  if (emit_only()) {
    C.cand += n;
    return "";
  }
  if (assemble) {
#ifdef ASMSIM_ASSEMBLER
    std::vector<char> code;
    std::string log;
    if (jit_compile_local(src, code, log)) {
      C.asmerror++;
      return "assembler: " + log.substr(0, 2000);
    }
#else
    return "built without the assembler (ASMSIM_ASSEMBLER)";
#endif
  }
  // random rows masked to each coordinate's width (mg_eval's layout); edge values now and then
  const uint32_t rows = low.coord_words;
  std::vector<uint32_t> soa((size_t)std::max<uint32_t>(rows, 1) * n, 0);
  uint64_t s = seed;
  for (uint32_t c = 0; c < low.coord_width.size(); c++) {
    const uint32_t w = low.coord_width[c], L = (w + 31) / 32;
    for (uint32_t j = 0; j < L; j++) {
      const uint32_t bits = std::min(32u, w - 32 * j);
      const uint32_t m = bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u);
      for (uint32_t i = 0; i < n; i++) {
        const uint64_t r = splitmix(s);
        uint32_t x = (uint32_t)r;
        switch ((r >> 32) & 7) {
          case 0: x = 0; break;
          case 1: x = (uint32_t)(r >> 40) & 3; break;
          case 2: x = 0xFFFFFFFFu; break;
          default: break;
        }
        soa[(size_t)(low.coord_row[c] + j) * n + i] = x & m;
      }
    }
  }
  std::vector<uint8_t> want(n);
  // the model read-back rows too (watch list kept: the kernel stores them, mg_jit_eval's watch_out)
  std::vector<uint32_t> want_w((size_t)sp.watch_words * n, 0);
  if (bv_eval_watch((const uint32_t*)prog.data(), prog.size() / 4, soa.data(), n, want.data(),
                    sp.watch_words ? want_w.data() : nullptr))
    return "C port eval failed";
  asmsim::Stats st;
  try {
    const asmsim::Module m = asmsim::parse(src);
    asmsim::Memory mem;
    std::vector<uint32_t> lay;
    uint64_t cols = n;
    if (tiled) {  // row r of candidate i at ((i / 64) * rows + r) * 64 + i % 64, whole blocks
      cols = (n + 63) / 64 * 64;
      lay.assign((size_t)std::max<uint32_t>(rows, 1) * cols, 0);
      for (uint32_t r = 0; r < rows; r++)
        for (uint32_t i = 0; i < n; i++) lay[((size_t)(i / 64) * rows + r) * 64 + i % 64] = soa[(size_t)r * n + i];
    } else {
      lay = soa;
    }
    const uint64_t sb = mem.add(lay.size() * 4, lay.data());
    const uint64_t ver = mem.add(n);
    const uint64_t wb = sp.watch_words ? mem.add((size_t)sp.watch_words * n * 4) : 0;
    // a loop-free solo kernel evaluates one 64-candidate group per workgroup (engine.hip mg_jit_eval_dev)
    const bool one_group = src.find("mgj_meta_eval_cpb:") != std::string::npos;
    const uint32_t nblk = one_group ? (uint32_t)((n + 63) / 64) : grid(n);
    std::vector<uint8_t> ka(64, 0);
    put64(ka, 0, sb);
    put64(ka, 8, n);
    put64(ka, 16, ver);
    put64(ka, 24, wb);
    put32(ka, 32, nblk);
    const uint64_t kb = mem.add(ka.size(), ka.data());
    asmsim::launch(m, "mgj_eval", mem, kb, nblk, &st);
    const uint8_t* got = mem.of(ver).data.data();
    for (uint32_t i = 0; i < n; i++)
      if (got[i] != want[i]) {
        C.mismatch++;
        char b[160];
        snprintf(b, sizeof b, "mgj_eval%s verdict of candidate %u: asm %u, C port %u", tiled ? " (tiled)" : "", i,
                 got[i], want[i]);
        return b;
      }
    if (sp.watch_words) {
      const uint32_t* gw = (const uint32_t*)mem.of(wb).data.data();
      for (size_t k = 0; k < want_w.size(); k++)
        if (gw[k] != want_w[k]) {
          C.mismatch++;
          char b[200];
          snprintf(b, sizeof b, "mgj_eval%s watch row %zu of candidate %zu: asm %08x, C port %08x", tiled ? " (tiled)" : "",
                   k / n, k % n, gw[k], want_w[k]);
          return b;
        }
    }
    if (getenv("ASMSIM_COUNT")) {  // as for the search launch: per candidate, and per program instruction
      printf("count eval: valu %.1f salu %.1f vmem %.2f nop %.1f branch %.1f waitcnt %.1f per candidate\n",
             64.0 * st.valu / n, 64.0 * st.salu / n, 64.0 * st.vmem / n, 64.0 * st.nop_slots / n,
             64.0 * st.branches / n, 64.0 * st.waitcnts / n);
      std::map<int, std::pair<uint64_t, uint64_t>> by;
      for (const auto& kv : st.valu_by_tag) by[kv.first].first = kv.second;
      for (const auto& kv : st.salu_by_tag) by[kv.first].second = kv.second;
      for (const auto& kv : by)
        printf("count tag %s: %.2f salu %.2f\n", m.tags[kv.first].c_str(), 64.0 * kv.second.first / n,
               64.0 * kv.second.second / n);
    }
  } catch (const asmsim::SimError& e) {
    C.simerror++;
    return "simulator: " + e.what;
  }
  C.valu += st.valu;
  C.cand += n;
  return "";
}

}  // namespace

int main() {
  Counts C;
  FILE* in = stdin;
  for (;;) {
    uint32_t kind, plen;
    if (!rd(in, &kind, 4)) break;
    if (!rd(in, &plen, 4)) return 3;
    std::vector<uint8_t> prog(plen);
    if (!rd(in, prog.data(), plen)) return 3;
    uint32_t gw;
    if (!rd(in, &gw, 4)) return 3;
    std::vector<uint32_t> gen;
    if (gw != 0xFFFFFFFFu) {
      gen.resize(gw);
      if (!rd(in, gen.data(), 4ull * gw)) return 3;
    }
    uint64_t seed, start;
    uint32_t count, flags;
    if (!rd(in, &seed, 8) || !rd(in, &start, 8) || !rd(in, &count, 4) || !rd(in, &flags, 4)) return 3;
    const uint64_t rec = C.records++;
    std::string why;
    const uint64_t before = C.outside;
    if (kind == 0) why = check_search(rec, prog, gen, seed, start, count, flags & 1, C);
    else why = check_eval(prog, seed, count, kind == 2, flags & 1, C);
    if (why.empty()) {
      if (C.outside == before) C.ok++;
    } else {
      printf("record %llu kind %u: %s\n", (unsigned long long)rec, kind, why.c_str());
      fflush(stdout);
    }
  }
  printf("records=%llu ok=%llu outside=%llu mismatch=%llu simerror=%llu asmerror=%llu valu=%llu cand=%llu\n",
         (unsigned long long)C.records, (unsigned long long)C.ok, (unsigned long long)C.outside,
         (unsigned long long)C.mismatch, (unsigned long long)C.simerror, (unsigned long long)C.asmerror,
         (unsigned long long)C.valu, (unsigned long long)C.cand);
  if (getenv("ASMSIM_TIMING"))
    fprintf(stderr, "emit %.2f s parse %.2f s sim %.2f s C port %.2f s\n", g_t[0], g_t[1], g_t[2], g_t[3]);
  return (C.mismatch || C.simerror || C.asmerror || C.records != C.ok + C.outside) ? 1 : 0;
}
