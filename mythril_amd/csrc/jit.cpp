// JIT specialisation: one lowered program -> straight-line HIP source ->
// hipRTC -> code object.  Every SSA value becomes scalar u32 limbs (v<id>_<j>) so
// LLVM allocates VGPRs; literals become immediates; the candidate generator is
// inlined per coordinate.  This removes the interpreter's per-instruction fetch,
// dispatch and value-file traffic (the dominant cost of k_run).
#include "jit.hpp"

#include <dlfcn.h>
#include <elf.h>
#include <signal.h>
#include <spawn.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <amd_comgr/amd_comgr.h>

#include <hip/hip_version.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>

#include <cerrno>
#include <cstdio>
#include <map>
#include <cstdlib>
#include <cstring>
#include <sstream>

namespace mg {

namespace {

const char* kPrelude =
#include "jit_prelude.inc"
    ;

inline uint32_t Lw(uint32_t w) { return (w + 31) / 32; }

struct Gen {
  const Lowered& P;
  const std::vector<GenSpec>* specs;
  const std::vector<uint32_t>* gconsts;
  std::ostringstream o;
  std::vector<int32_t> def;  // value id -> index of its defining instruction in P.vcode (-1: none)
  Gen(const Lowered& p, const std::vector<GenSpec>* s, const std::vector<uint32_t>* g)
      : P(p), specs(s), gconsts(g), def(p.vwidth.size(), -1) {
    for (size_t k = 0; k < P.vcode.size(); k++)
      if (P.vcode[k].dst != MG_NONE && P.vcode[k].dst < def.size() && def[P.vcode[k].dst] < 0)
        def[P.vcode[k].dst] = (int32_t)k;
  }
  const Instr* def_of(uint32_t id) const { return def[id] >= 0 ? &P.vcode[def[id]] : nullptr; }
  // literal limbs of a value defined by K_CONST (else nullptr)
  const uint32_t* lit(uint32_t id) const {
    const Instr* d = def_of(id);
    return (d && d->op == K_CONST) ? &P.consts[d->p0] : nullptr;
  }

  // A dictionary of n entries of a coordinate at most 32 bits wide whose n*width bits fit in 64 is
  // packed into one 64-bit literal: entry `idx` is a shift and a mask in VGPRs instead of a per-lane
  // gather from gconsts (one VMEM instruction per coordinate and candidate; the C2 query has 124
  // such byte coordinates).  Returns "" when the dictionary does not fit.
  std::string packed_dict(uint32_t off, uint32_t n, uint32_t w, const std::string& idx) const {
    if (w > 32 || n == 0 || (uint64_t)n * w > 64) return "";
    uint64_t pack = 0;
    const uint64_t m = w == 64 ? ~0ull : ((1ull << w) - 1ull);
    for (uint32_t e = 0; e < n; e++) pack |= ((uint64_t)(*gconsts)[off + e] & m) << (e * w);
    std::ostringstream t;
    t << "(uint32_t)((0x" << std::hex << pack << "ull >> (" << idx << " * " << std::dec << w << "u)) & 0x" << std::hex
      << m << "ull)";
    return t.str();
  }

  // Dictionary tables of the generator, staged in LDS by the search/gen kernels' prologue: a
  // per-lane gather of a 256-bit entry from global memory moves 32 B per lane through the
  // vector L1 (measured on C2: two 3-entry DICT coordinates cost a quarter of the kernel time),
  // LDS serves it at twice the bandwidth and nothing else in the kernel uses LDS.  Limbs that
  // are the same in every entry are literals and are not read at all.
  std::map<uint32_t, uint32_t> dict_lds;  // gconsts offset of a table -> LDS word offset
  std::map<uint32_t, uint32_t> dict_n;    // gconsts offset of a table -> entries
  uint32_t lds_words = 0;
  static constexpr uint32_t kDictLdsWords = 4096;  // 16 KiB per 256-lane block
  // dictionaries up to this many entries are selects, not gathers (MYTHGPU_JIT_SELECT_DICT, default 4)
  static uint32_t select_dict_max() {
    static const uint32_t n = [] {
      const char* g = getenv("MYTHGPU_JIT_SELECT_DICT");
      return g ? (uint32_t)atoi(g) : 4u;
    }();
    return n;
  }

  // Staged tables in quads of limbs: limbs 4q .. 4q+3 of entry e at word base + 4qn + 4e (the top quad
  // padded), read as one 16-byte load where two or more of its limbs vary — ds_read_b128 moves 16
  // bytes per lane in 4 LDS cycles, four times a ds_read_b32's bytes per cycle (MI355X_MICROARCH.md
  // §LDS).  (Pairs were tried first: LLVM merges two 8-byte loads into ds_read2_b64, which takes twice
  // a ds_read_b64's cycles.)  MYTHGPU_JIT_DICT_PAIRS=0: limb-major ([limb][entry])
  static bool dict_pairs() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_DICT_PAIRS");
      return !(g && g[0] == '0');
    }();
    return on;
  }
  void plan_dict_lds() {
    dict_lds.clear();
    dict_n.clear();
    lds_words = 0;
    // on by default since the tables are limb-major (MYTHGPU_JIT_DICT_LDS=0: per-lane gathers from
    // global memory): C1 +40 %, C2 +3.7 %, C4 +2.5 %, C3 -8 % (profiles/r03_ab_dict_lds.jsonl)
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_DICT_LDS");
      return !(g && g[0] == '0');
    }();
    if (!specs || !on) return;
    // only when several coordinates gather from tables: with one or two (C3) the per-block staging
    // and the LDS reads cost more than the gathers they replace (C3 -8 %, profiles/r03_ab_dict_lds.jsonl)
    uint32_t gathering = 0;
    for (uint32_t c = 0; c < specs->size(); c++) {
      const GenSpec& sp = (*specs)[c];
      const uint32_t kind = sp.kind & 0xFFu, n = sp.p[1];
      const bool dict = kind == MG_GEN_DICT || (kind == MG_GEN_MIXED && n && (sp.p[2] >> 16));
      if (dict && c < P.coord_width.size() && n > select_dict_max() && !coord_dead(c) &&
          packed_dict(sp.p[0], n, P.coord_width[c], "e").empty())
        gathering++;
    }
    if (gathering < 3) return;
    for (uint32_t c = 0; c < specs->size(); c++) {
      const GenSpec& sp = (*specs)[c];
      const uint32_t kind = sp.kind & 0xFFu;
      const uint32_t n = sp.p[1], off = sp.p[0];
      const bool dict = kind == MG_GEN_DICT || (kind == MG_GEN_MIXED && n && (sp.p[2] >> 16));
      if (!dict || n == 0 || c >= P.coord_width.size() || coord_dead(c)) continue;
      const uint32_t w = P.coord_width[c], L = Lw(w);
      if (!packed_dict(off, n, w, "e").empty() || dict_lds.count(off) || n <= select_dict_max()) continue;
      const uint32_t need = dict_pairs() ? n * ((L + 3u) & ~3u) : (n * L + 3u) & ~3u;  // 16-B aligned tables
      if (lds_words + need > kDictLdsWords) continue;
      dict_lds[off] = lds_words;
      dict_n[off] = n;
      lds_words += need;
    }
  }

  // Tables gathered from global memory are baked into the code object, entry-major with each
  // entry on a 16-B boundary, so a lane reads a 256-bit entry with two 16-B loads instead of one
  // 4-B load per limb: a per-lane gather is one texture-path request per lane and instruction,
  // and eight of them per entry kept the path busy (C3: two 74-entry tables of 256-bit words,
  // frac 0.31 with 2.8 gathers per wave and half the wave cycles waiting).
  // MYTHGPU_JIT_DICT_VEC=0: per-limb gathers from the generator blob.
  std::map<uint32_t, uint32_t> dict_gv;  // gconsts offset of a table -> word offset in mg_gd
  std::map<uint32_t, uint32_t> dict_gv_stride;
  std::vector<uint32_t> gd;              // the baked tables
  void plan_dict_gv() {
    dict_gv.clear();
    dict_gv_stride.clear();
    gd.clear();
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_DICT_VEC");
      return !(g && g[0] == '0');
    }();
    if (!specs || !on) return;
    const auto& G = *gconsts;
    for (uint32_t c = 0; c < specs->size(); c++) {
      const GenSpec& sp = (*specs)[c];
      const uint32_t kind = sp.kind & 0xFFu;
      const uint32_t n = sp.p[1], off = sp.p[0];
      const bool dict = kind == MG_GEN_DICT || (kind == MG_GEN_MIXED && n && (sp.p[2] >> 16));
      if (!dict || n == 0 || c >= P.coord_width.size() || coord_dead(c)) continue;
      const uint32_t w = P.coord_width[c], L = Lw(w);
      if (L < 2 || dict_gv.count(off) || dict_lds.count(off) || n <= select_dict_max()) continue;
      if ((size_t)off + (size_t)n * L > G.size()) continue;
      const uint32_t S = L == 2 ? 2u : (L + 3u) & ~3u;
      if (gd.size() + (size_t)n * S > (1u << 16)) continue;
      dict_gv[off] = (uint32_t)gd.size();
      dict_gv_stride[off] = S;
      for (uint32_t e = 0; e < n; e++)
        for (uint32_t j = 0; j < S; j++) gd.push_back(j < L ? G[off + e * L + j] : 0u);
    }
  }

  // the baked tables, at namespace scope before the kernels
  void emit_dict_gv_table() {
    if (gd.empty()) return;
    o << "__device__ __attribute__((aligned(16))) const uint32_t mg_gd[" << gd.size() << "] = {";
    for (size_t i = 0; i < gd.size(); i++) o << (i % 8 ? "" : "\n  ") << hex(gd[i]) << ",";
    o << "\n};\n";
  }
  uint32_t gv_tmp = 0;

  // kernel prologue: copy the planned tables into LDS (all 256 lanes), then a block barrier
  void emit_dict_prologue() {
    if (!lds_words) return;
    o << "  __shared__ __attribute__((aligned(16))) uint32_t mg_dict[" << lds_words << "];\n";
    std::map<uint32_t, uint32_t> len;  // table -> words (n * L)
    for (uint32_t c = 0; c < specs->size(); c++) {
      const GenSpec& sp = (*specs)[c];
      auto it = dict_lds.find(sp.p[0]);
      const uint32_t kind = sp.kind & 0xFFu;
      if (it == dict_lds.end() || c >= P.coord_width.size()) continue;
      if (!(kind == MG_GEN_DICT || kind == MG_GEN_MIXED)) continue;
      len[sp.p[0]] = std::max(len[sp.p[0]], sp.p[1] * Lw(P.coord_width[c]));
    }
    // limb-major ([limb][entry]): lanes that drew different entries read different banks (entry-major,
    // a 256-bit table put every lane's limb j in one of 4 banks: 16-way conflicts)
    for (const auto& kv : len) {
      const uint32_t n = dict_n.at(kv.first), L = kv.second / std::max(n, 1u);
      if (dict_pairs())
        o << "  for (uint32_t i = tid; i < " << kv.second << "u; i += 256u) mg_dict[" << dict_lds.at(kv.first)
          << "u + ((i % " << L << "u) & ~3u) * " << n << "u + 4u * (i / " << L << "u) + ((i % " << L
          << "u) & 3u)] = gconsts[" << kv.first << "u + i];\n";
      else
        o << "  for (uint32_t i = tid; i < " << kv.second << "u; i += 256u) mg_dict[" << dict_lds.at(kv.first)
          << "u + (i % " << L << "u) * " << n << "u + i / " << L << "u] = gconsts[" << kv.first << "u + i];\n";
    }
    o << "  __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"workgroup\");\n"
         "  __builtin_amdgcn_s_barrier();\n"
         "  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"workgroup\");\n";
  }

  // limbs of entry `idx` of the n-entry table at gconsts offset `off` (coordinate width w)
  template <class Lim>
  void dict_limbs(uint32_t off, uint32_t n, uint32_t w, const std::string& idx, const Lim& lim, const char* ind) {
    const uint32_t L = Lw(w);
    const std::string packed = packed_dict(off, n, w, idx);
    if (!packed.empty()) {
      for (uint32_t j = 0; j < L; j++) o << ind << lim(j) << " = " << (j ? std::string("0u") : packed) << ";\n";
      return;
    }
    const auto& G = *gconsts;
    auto lds = dict_lds.find(off);
    auto gv = dict_gv.find(off);
    std::vector<std::string> gvl(L);  // limb j of the entry read by vector loads from mg_gd
    if (gv != dict_gv.end() && n > select_dict_max()) {
      const uint32_t S = dict_gv_stride.at(off), q = S == 2 ? 2u : 4u;
      for (uint32_t b = 0; b < L; b += q) {
        bool need = false;
        for (uint32_t j = b; j < std::min(L, b + q) && !need; j++)
          for (uint32_t e = 1; e < n && !need; e++) need = G[off + e * L + j] != G[off + j];
        if (!need) continue;
        const std::string t = "mg_gq" + std::to_string(gv_tmp++);
        o << ind << "const u32x" << q << " " << t << " = *(const u32x" << q << "*)(mg_gd + " << gv->second + b
          << "u + " << idx << " * " << S << "u);\n";
        static const char* comp = "xyzw";
        for (uint32_t j = b; j < std::min(L, b + q); j++) gvl[j] = t + "." + comp[j - b];
      }
    }
    auto varies = [&](uint32_t j) {
      for (uint32_t e = 1; e < n; e++)
        if (G[off + e * L + j] != G[off + j]) return true;
      return false;
    };
    std::vector<std::string> pl(L);  // limb j from a quad load of the LDS copy
    if (lds != dict_lds.end() && dict_pairs() && n > select_dict_max())
      for (uint32_t b = 0; b < L; b += 4) {
        uint32_t k = 0;
        for (uint32_t j = b; j < std::min(L, b + 4); j++) k += varies(j) && gvl[j].empty();
        if (k < 2) continue;
        const std::string t = "mg_gq" + std::to_string(gv_tmp++);
        o << ind << "const u32x4 " << t << " = *(const u32x4*)(mg_dict + " << lds->second + b * n << "u + 4u * " << idx
          << ");\n";
        static const char* comp = "xyzw";
        for (uint32_t j = b; j < std::min(L, b + 4); j++) pl[j] = t + "." + comp[j - b];
      }
    for (uint32_t j = 0; j < L; j++) {
      bool same = true;
      for (uint32_t e = 1; e < n && same; e++) same = G[off + e * L + j] == G[off + j];
      std::string v;
      if (same) {
        v = hex(G[off + j]);
      } else if (n <= select_dict_max()) {
        // a select over the entries' literals (v_cndmask): a per-lane gather is one VMEM
        // instruction per limb, and the CU's one texture path serves its four SIMDs at a
        // fraction of their VALU issue rate
        v = hex(G[off + (n - 1) * L + j]);
        for (int32_t e = (int32_t)n - 2; e >= 0; e--)
          v = "(" + idx + " == " + std::to_string(e) + "u ? " + hex(G[off + e * L + j]) + " : " + v + ")";
      } else if (!gvl[j].empty()) v = gvl[j];
      else if (!pl[j].empty()) v = pl[j];
      else if (lds != dict_lds.end() && dict_pairs())
        v = "mg_dict[" + std::to_string(lds->second + (j & ~3u) * n + (j & 3u)) + "u + 4u * " + idx + "]";
      else if (lds != dict_lds.end()) v = "mg_dict[" + std::to_string(lds->second + j * n) + "u + " + idx + "]";
      else v = "gconsts[" + std::to_string(off + j) + "u + " + idx + " * " + std::to_string(L) + "u]";
      o << ind << lim(j) << " = " << v << ";\n";
    }
  }

  // Spec-specialised GEN3 generator for coordinate c (the same function of (seed, index, c)
  // as gen_coord in engine.hip and gen_value in oracle/bveval.c).  Writes L limbs into
  // `out`_j.  A MIXED coordinate's alternative comes from the group key (SGPRs), so the
  // alternatives are scalar branches: a lane computes only the one its wave chose.
  // Lane-parallel group keys (MYTHGPU_JIT_LANE_KEYS=1; off by default: measured C1 -1 %, C2 -6 %,
  // C3 +1.7 %, C4 +0.6 %, profiles/r03_ab_lanekeys.jsonl — the scalar unit was not what bounds C1/C3).  Per group of 64 candidates the
  // scalar unit would hash the group key G (fmix64: ~20 SALU) and every MIXED coordinate's choice
  // word ws (3 SALU each); with four SIMDs sharing the CU's scalar unit, small query kernels (C1,
  // C3) are scalar-bound.  Instead lane l of a wave hashes G of the wave's (k + l)-th group once
  // per 64 groups (VALU), and per group lane j computes ws of the j-th MIXED coordinate (3 VALU for
  // all of them); G and each ws are then one v_readlane each.  Same values as gen_keys / gwsel.
  std::map<uint32_t, uint32_t> ws_slot;  // MIXED coordinate -> lane of wsv holding its ws
  static bool lane_keys() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_LANE_KEYS");
      return g && g[0] == '1';
    }();
    return on;
  }
  void plan_ws_slots() {
    ws_slot.clear();
    if (!specs || !lane_keys()) return;
    for (uint32_t c = 0; c < specs->size() && ws_slot.size() < 64; c++)
      if (((*specs)[c].kind & 0xFFu) == MG_GEN_MIXED && !coord_dead(c)) ws_slot[c] = (uint32_t)ws_slot.size();
  }
  // a coordinate no search can read: LAZY, or neither read by the program nor a COPY source of one
  std::vector<char> reach;
  bool coord_dead(uint32_t c) {
    if (reach.empty()) {
      reach.assign(specs->size(), 0);
      std::vector<uint32_t> st;
      for (const Instr& in : P.vcode)
        if (in.op == K_COORD && in.p0 < reach.size() && !reach[in.p0]) { reach[in.p0] = 1; st.push_back(in.p0); }
      while (!st.empty()) {
        const uint32_t x = st.back();
        st.pop_back();
        const GenSpec& sp = (*specs)[x];
        if ((sp.kind & 0xFFu) == MG_GEN_MIXED && sp.p[3] != MG_NONE && (sp.p[2] & 0xFFFFu) && !reach[sp.p[3]]) {
          reach[sp.p[3]] = 1;
          st.push_back(sp.p[3]);
        }
      }
    }
    return !reach[c];
  }
  // kernel prologue: the per-lane salt of the choice word (lane j: coordinate of slot j)
  void emit_ws_salt() {
    if (!lane_keys()) return;
    o << "  uint32_t gkv_lo = 0u, gkv_hi = 0u;  // lane l: the group key of the wave's group kk + l\n";
    if (ws_slot.empty()) return;
    std::vector<uint32_t> salt(ws_slot.size());
    for (const auto& kv : ws_slot) salt[kv.second] = kv.first * 0x9E3779B9u + 0xFFFEu * 0x85EBCA6Bu + 0x27D4EB2Fu;
    std::string e = hex(salt.back());
    for (int32_t j = (int32_t)salt.size() - 2; j >= 0; j--) e = "(lane == " + std::to_string(j) + "u ? " + hex(salt[j]) + " : " + e + ")";
    o << "  const uint32_t wsalt = " << e << ";\n";
  }
  // group prologue: G for this group (from the lanes' cache, refilled every 64 groups) and wsv
  void emit_group_keys(const char* kk, const char* g, const char* gstride) {
    if (!lane_keys()) {
      o << "  const uint64_t G = fmix64((gbase >> 6) ^ sg);\n";
      return;
    }
    o << "  if ((" << kk << " & 63u) == 0u) { const uint64_t Gx = fmix64(((a0 >> 6) + " << g << " + (uint64_t)lane * "
      << gstride << ") ^ sg); gkv_lo = (uint32_t)Gx; gkv_hi = (uint32_t)(Gx >> 32); }\n"
         "  const uint64_t G = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)gkv_hi, (int)(" << kk << " & 63u)) << 32) | "
         "(uint32_t)__builtin_amdgcn_readlane((int)gkv_lo, (int)(" << kk << " & 63u));\n";
    if (!ws_slot.empty())
      o << "  const uint32_t wsv = (((uint32_t)G ^ wsalt) * 0x9E3779B1u) + (uint32_t)(G >> 32);\n";
  }
  std::map<uint32_t, std::string> coord_var;  // coordinate -> prefix of its generated (final) limbs
  int tmp_id = 0;

  // Dictionary gathers one group ahead (search kernel).  A MIXED coordinate whose DICT alternative
  // gathers from global memory loads its entry where its value is needed, so a wave waits out the
  // load every group it chose DICT (C3: two 256-bit gathers from a 74-entry table, half the wave
  // cycles waiting).  Instead the group loop carries the next group's key: at the top of group k
  // the wave hashes group k+1's choice word and, if it chose DICT, its lanes' entries and issues
  // the loads; group k's own entries arrived during group k-1.  Same values (a pure function of
  // group and coordinate), one fmix64 per group as before.  Opt-in (MYTHGPU_JIT_PREFETCH=1): C3
  // measured 12 % SLOWER with it (profiles/r03_ab_prefetch.jsonl) — the loop-carried entries cost a
  // register copy per limb and group, and the gathers were not what C3 waits on.
  std::vector<uint32_t> pf;  // coordinates prefetched
  bool pf_active = false;    // emitting the search kernel's body: read the prefetched registers
  void plan_prefetch() {
    pf.clear();
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_PREFETCH");
      return g && g[0] == '1';
    }();
    if (!specs || !on || lane_keys()) return;
    for (uint32_t c = 0; c < specs->size() && c < P.coord_width.size(); c++) {
      const GenSpec& sp = (*specs)[c];
      if ((sp.kind & 0xFFu) != MG_GEN_MIXED || coord_dead(c)) continue;
      const uint32_t pd = sp.p[1] ? (sp.p[2] >> 16) : 0u, n = sp.p[1], w = P.coord_width[c];
      if (!pd || n <= select_dict_max() || Lw(w) > 8 || dict_lds.count(sp.p[0])) continue;
      if (!packed_dict(sp.p[0], n, w, "e").empty()) continue;
      pf.push_back(c);
    }
  }
  void emit_prefetch_decls() {
    for (uint32_t c : pf) {
      o << "  uint32_t pfh" << c << " = 0u";
      for (uint32_t j = 0; j < Lw(P.coord_width[c]); j++) o << ", pf" << c << "_" << j << " = 0u";
      o << ";\n";
    }
  }
  // the loads for the group whose key is Gn
  void emit_prefetch(const char* Gn) {
    if (pf.empty()) return;
    o << "  { GKeys kn; { const uint64_t K = " << Gn << " ^ LK;\n"
         "    kn.klo = (uint32_t)K; kn.khi = (uint32_t)(K >> 32); kn.kf = kn.klo ^ (kn.klo >> 16); kn.glo = (uint32_t)" << Gn
      << "; kn.ghi = (uint32_t)(" << Gn << " >> 32); }\n";
    for (uint32_t c : pf) {
      const GenSpec& sp = (*specs)[c];
      const uint32_t pc = sp.p[3] != MG_NONE ? (sp.p[2] & 0xFFFFu) : 0u;
      const uint32_t pd = sp.p[2] >> 16;
      const uint32_t lo = pc << 16, hi = pc + pd;
      o << "    { const uint32_t wsn = gwsel(kn, " << c << "u);\n"
        << "      if (" << (pc ? "wsn >= " + hex(lo) : std::string("true")) << " && "
        << (hi >= 65536u ? std::string("true") : "wsn < " + hex(hi << 16)) << ") {\n"
        << "        pfh" << c << " = grnd(kn, " << c << "u, 0xFFFFu);\n"
        << "        const uint32_t e = ((pfh" << c << " >> 16) * " << sp.p[1] << "u) >> 16;\n";
      const std::string pre = "pf" + std::to_string(c) + "_";
      dict_limbs(sp.p[0], sp.p[1], P.coord_width[c], "e", [&](uint32_t j) { return pre + std::to_string(j); },
                 "        ");
      o << "      } }\n";
    }
    o << "  }\n";
  }
  // at the top of a group: this group's prefetched values, before the next group's loads overwrite them
  void emit_prefetch_take() {
    for (uint32_t c : pf) {
      o << "  const uint32_t ch" << c << " = pfh" << c;
      for (uint32_t j = 0; j < Lw(P.coord_width[c]); j++) o << ", cv" << c << "_" << j << " = pf" << c << "_" << j;
      o << ";\n";
    }
  }
  bool prefetched(uint32_t c) const { return pf_active && std::find(pf.begin(), pf.end(), c) != pf.end(); }

  std::string gen_coord_value(uint32_t c) {
    auto it = coord_var.find(c);
    if (it != coord_var.end()) return it->second;
    // a copy source with no K_COORD of its own: generate it into temporaries
    const std::string pre = "cg" + std::to_string(c) + "_" + std::to_string(tmp_id++);
    const uint32_t L = Lw(P.coord_width[c]);
    o << "  uint32_t";
    for (uint32_t j = 0; j < L; j++) o << (j ? ", " : " ") << pre << "_" << j;
    o << ";\n";
    gen_value(c, pre);
    return pre;
  }

  // UNIFORM raw limbs (mythgpu.h GEN3): u0, u1 hashed, u_j = gext(u_{j-1}, u_{j-2}, j); limb j of
  // the value is u_j masked to the low `bits` bits of the value
  template <class Lim>
  void uniform_limbs(const std::string& C, uint32_t L, uint32_t bits, const Lim& lim, const char* ind) {
    const uint32_t need = std::min(L, (bits + 31) / 32);  // raw limbs that reach the value
    const std::string u = "u" + std::to_string(tmp_id++) + "_";
    for (uint32_t j = 0; j < need; j++) {
      o << ind << "const uint32_t " << u << j << " = "
        << (j < 2 ? "grnd(ky, " + C + ", " + std::to_string(j) + "u)"
                  : "gext(" + u + std::to_string(j - 1) + ", " + u + std::to_string(j - 2) + ", " + std::to_string(j) + "u)")
        << ";\n";
    }
    for (uint32_t j = 0; j < L; j++) {
      const uint32_t lo = 32 * j;
      const uint32_t m = lo >= bits ? 0u : (bits - lo >= 32 ? 0xFFFFFFFFu : ((1u << (bits - lo)) - 1u));
      std::string e = u + std::to_string(j);
      if (m == 0) e = "0u";
      else if (m != 0xFFFFFFFFu) e = "(" + e + " & " + hex(m) + ")";
      o << ind << lim(j) << " = " << e << ";\n";
    }
  }

  void gen_value(uint32_t c, const std::string& out) {
    const GenSpec sp = (*specs)[c];
    const uint32_t fix = sp.kind >> 8;  // 1 + const offset of (mask, value) limbs, 0: none
    const uint32_t kind = sp.kind & 0xFFu;
    const uint32_t width = P.coord_width[c];
    const uint32_t L = Lw(width);
    const std::string C = std::to_string(c) + "u";
    auto lim = [&](uint32_t j) { return out + "_" + std::to_string(j); };
    const auto& G = *gconsts;
    o << "  {\n";
    switch (kind) {
      case MG_GEN_MIXED: {
        const uint32_t pc = sp.p[3] != MG_NONE ? (sp.p[2] & 0xFFFFu) : 0u;
        const uint32_t pd = sp.p[1] ? (sp.p[2] >> 16) : 0u;
        const uint32_t ps = sp.p[4] & 0xFFFFu;
        const uint32_t small_bits = std::min(width, sp.p[4] >> 16);
        const bool narrow = width <= MG_GEN_NARROW_BITS;
        // the alternative is s = ws >> 16 (wave-uniform, SGPRs): s < T  <=>  ws < T << 16, so each
        // test is one scalar compare; h is hashed only in the branches that read it
        {
          auto sl = ws_slot.find(c);
          if (sl != ws_slot.end())  // the choice word computed lane-parallel for the group (lane_keys)
            o << "  const uint32_t ws = (uint32_t)__builtin_amdgcn_readlane((int)wsv, " << sl->second << ");\n";
          else
            o << "  const uint32_t ws = gwsel(ky, " << C << ");\n";
        }
        const std::string hdecl = "const uint32_t h = grnd(ky, " + C + ", 0xFFFFu);";
        auto below = [&](uint32_t T) {
          return T >= 65536u ? std::string("true") : "ws < " + hex(T << 16);
        };
        // uniform / small limbs (narrow: from h)
        auto uni = [&](uint32_t bits) {
          if (narrow) {
            o << "    " << hdecl << "\n";
            for (uint32_t j = 0; j < L; j++) {
              const uint32_t m = j ? 0u : (bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u));
              o << "    " << lim(j) << " = " << (m ? "(h & " + hex(m & 0xFFFFu) + ")" : std::string("0u")) << ";\n";
            }
            return;
          }
          uniform_limbs(C, L, bits, lim, "    ");
        };
        // +/-(1 + (h & 1)) on COPY / DICT as ONE carry chain over the sign-extended step, when the
        // low half of ws is below P(delta); emitted inside the COPY and DICT branches
        auto delta = [&](bool h_known) {
          if (!sp.p[5]) return;
          o << "    if ((ws & 0xFFFFu) < " << sp.p[5] << "u) {" << (h_known ? "" : " " + hdecl)
            << " const uint32_t mag = 1u + (h & 1u); const bool sb = (h >> 1) & 1u;"
            << " const uint32_t a0 = sb ? 0u - mag : mag, ah = sb ? 0xFFFFFFFFu : 0u; uint32_t cy = 0u;";
          // the high limbs change only in a lane whose low-limb carry differs from the step's sign
          // (x + 0 + 0 and x + ~0 + 1 are x): the rest of the chain runs only when some lane of the
          // wave needs it (MYTHGPU_JIT_DELTA_SKIP=0: always)
          static const bool skip = [] {
            const char* g = getenv("MYTHGPU_JIT_DELTA_SKIP");
            return !(g && g[0] == '0');
          }();
          for (uint32_t j = 0; j < L; j++) {
            if (j == 1 && skip) o << " if (__ballot(cy != (uint32_t)sb)) {";
            o << " " << lim(j) << " = mg_addc(" << lim(j) << ", " << (j ? "ah" : "a0") << ", cy, &cy);";
          }
          if (L > 1 && skip) o << " }";
          o << " (void)cy; (void)ah; }\n";
        };
        // mask + clamp, emitted at the end of EACH branch: what a branch knows about its limbs
        // (SMALL: the high limbs are zero; DICT: limbs equal in every entry are literals) folds
        // the clamp test there
        auto finish = [&]() {
          if (width & 31) o << "    " << lim(L - 1) << " &= " << hex(topmask(width)) << ";\n";
          if (!sp.p[6]) return;
          const uint32_t r = sp.p[6] - 1;
          const uint32_t span = G[r + L];
          const uint32_t k = reach_limbs(&G[r], L, span ? span - 1u : 0xFFFFFFFFull, 0);
          o << "    { uint32_t br = 0u, hz = 0u, t0;";
          for (uint32_t j = 0; j < L; j++) {
            if (j == 0) o << " t0 = mg_subc(" << lim(0) << ", " << hex(G[r]) << ", br, &br);";
            else o << " hz |= mg_subc(" << lim(j) << ", " << hex(G[r + j]) << ", br, &br);";
          }
          o << " if (br | hz" << (span ? " | (uint32_t)(t0 >= " + hex(span) + ")" : std::string("")) << ") {"
            << " const uint32_t off = " << (span ? "(uint32_t)(((uint64_t)" + lim(0) + " * " + std::to_string(span) + "ull) >> 32)" : lim(0))
            << "; uint32_t cy = 0u;";
          for (uint32_t j = 0; j < L; j++) {
            if (j < k) o << " " << lim(j) << " = mg_addc(" << hex(G[r + j]) << ", " << (j ? "0u" : "off") << ", cy, &cy);";
            else o << " " << lim(j) << " = " << hex(G[r + j]) << ";";
          }
          o << " (void)cy; } }\n";
        };
        bool first = true;
        auto branch = [&](const std::string& cond) {
          o << (first ? "  if (" : "  } else if (") << cond << ") {\n";
          first = false;
        };
        if (pc) {
          branch(below(pc));
          std::string src;
          auto cv = coord_var.find(sp.p[3]);
          if (cv != coord_var.end()) {
            src = cv->second;
          } else {
            // a copy source the program does not read before this point: generated only by the
            // waves that take this branch, into temporaries scoped to it
            const auto saved = coord_var;
            src = gen_coord_value(sp.p[3]);
            coord_var = saved;
          }
          for (uint32_t j = 0; j < L; j++) o << "    " << lim(j) << " = " << src << "_" << j << ";\n";
          delta(false);
          finish();
        }
        if (pd) {
          branch(below(pc + pd));
          if (prefetched(c)) {  // loaded one group ahead (plan_prefetch)
            o << "    const uint32_t h = ch" << c << ";\n";
            for (uint32_t j = 0; j < L; j++) o << "    " << lim(j) << " = cv" << c << "_" << j << ";\n";
          } else {
            o << "    " << hdecl << "\n";
            // MYTHGPU_JIT_DICT_SPREAD=1 (diagnostic: WRONG verdicts): lane l of a 32-lane LDS group reads
            // entry l, so the dictionary reads have no bank conflicts — what the conflicts cost.  Taken
            // only together with MYTHGPU_UNSAFE_DIAGNOSTICS=1 (a profiling run's explicit opt-in); the
            // switch alone is ignored with a warning, so it cannot leak into a user's searches
            static const bool spread = [] {
              const char* g = getenv("MYTHGPU_JIT_DICT_SPREAD");
              if (!(g && g[0] == '1')) return false;
              const char* u = getenv("MYTHGPU_UNSAFE_DIAGNOSTICS");
              if (u && u[0] == '1') {
                fprintf(stderr, "mythgpu: MYTHGPU_JIT_DICT_SPREAD=1: O3 search kernels give WRONG verdicts (timing only)\n");
                return true;
              }
              fprintf(stderr, "mythgpu: MYTHGPU_JIT_DICT_SPREAD ignored (needs MYTHGPU_UNSAFE_DIAGNOSTICS=1)\n");
              return false;
            }();
            if (spread && sp.p[1] >= 32 && dict_lds.count(sp.p[0]))
              o << "    const uint32_t e = lane & 31u; (void)h;\n";
            else
              o << "    const uint32_t e = ((h >> 16) * " << sp.p[1] << "u) >> 16;\n";
            dict_limbs(sp.p[0], sp.p[1], width, "e", lim, "    ");
          }
          delta(true);
          finish();
        }
        if (ps) {
          branch(below(pc + pd + ps));
          uni(small_bits);
          finish();
        }
        if (first) {
          uni(width);
          finish();
        } else {
          o << "  } else {\n";
          uni(width);
          finish();
          o << "  }\n";
        }
        break;
      }
      case MG_GEN_DICT: {
        o << "  const uint32_t e = ((grnd(ky, " << C << ", 0xFFFFu) >> 16) * " << sp.p[1] << "u) >> 16;\n";
        dict_limbs(sp.p[0], sp.p[1], width, "e", lim, "  ");
        break;
      }
      case MG_GEN_RANGE: {
        o << "  const uint32_t r = grnd(ky, " << C << ", 0u); const uint32_t off = "
          << (sp.p[1] ? ("(uint32_t)(((uint64_t)r * " + std::to_string(sp.p[1]) + "ull) >> 32)") : std::string("r"))
          << "; uint32_t cy = 0u;\n";
        const uint32_t k = reach_limbs(&G[sp.p[0]], L, sp.p[1] ? sp.p[1] - 1u : 0xFFFFFFFFull, 0);
        for (uint32_t j = 0; j < L; j++) {
          if (j < k)
            o << "  " << lim(j) << " = mg_addc(" << hex(G[sp.p[0] + j]) << ", " << (j ? "0u" : "off") << ", cy, &cy);\n";
          else
            o << "  " << lim(j) << " = " << hex(G[sp.p[0] + j]) << ";\n";
        }
        o << "  (void)cy;\n";
        break;
      }
      case MG_GEN_ALIGNED: {
        o << "  const uint32_t r = grnd(ky, " << C << ", 0u); const uint64_t m = "
          << (sp.p[2] ? ("(((uint64_t)r * " + std::to_string(sp.p[2]) + "ull) >> 32)") : std::string("(uint64_t)r"))
          << "; uint32_t cy = 0u;\n";
        const int32_t sh = (int32_t)sp.p[1];
        const uint32_t k = reach_limbs(&G[sp.p[0]], L, sp.p[2] ? sp.p[2] - 1u : 0xFFFFFFFFull, (uint32_t)sh);
        static const bool wide = [] {  // MYTHGPU_JIT_ALIGNED64=0: the limb-wise carry chain
          const char* g = getenv("MYTHGPU_JIT_ALIGNED64");
          return !(g && g[0] == '0');
        }();
        if (wide && k == 2 && L >= 2 && sh >= 0 && sh < 32) {
          // the offset reaches two limbs: one 64-bit (m << sh) + base (v_lshl_add_u64 / v_mad_u64_u32)
          const uint64_t base = ((uint64_t)G[sp.p[0] + 1] << 32) | G[sp.p[0]];
          o << "  { const uint64_t s64 = (m << " << sh << ") + " << base << "ull;\n";
          o << "  " << lim(0) << " = (uint32_t)s64;\n  " << lim(1) << " = (uint32_t)(s64 >> 32); }\n";
          for (uint32_t j = 2; j < L; j++) o << "  " << lim(j) << " = " << hex(G[sp.p[0] + j]) << ";\n";
          o << "  (void)cy;\n";
          break;
        }
        for (uint32_t j = 0; j < L; j++) {
          const int32_t bit0 = (int32_t)(j * 32) - sh;
          std::string mw;
          if (bit0 <= -32 || bit0 >= 64) mw = "0u";
          else if (bit0 < 0) mw = "(uint32_t)(m << " + std::to_string(-bit0) + ")";
          else mw = "(uint32_t)(m >> " + std::to_string(bit0) + ")";
          if (j < k) o << "  " << lim(j) << " = mg_addc(" << hex(G[sp.p[0] + j]) << ", " << mw << ", cy, &cy);\n";
          else o << "  " << lim(j) << " = " << hex(G[sp.p[0] + j]) << ";\n";
        }
        o << "  (void)cy;\n";
        break;
      }
      case MG_GEN_FIXED:
        for (uint32_t j = 0; j < L; j++) o << "  " << lim(j) << " = " << hex(G[sp.p[0] + j]) << ";\n";
        break;
      default:  // UNIFORM / LAZY
        uniform_limbs(C, L, 32 * L, lim, "  ");
        break;
    }
    if (width & 31) o << "  " << lim(L - 1) << " &= " << hex(topmask(width)) << ";\n";
    if (fix) {
      // fixed bits are literals here: (v & ~mask) | value
      const uint32_t f = fix - 1;
      for (uint32_t j = 0; j < L; j++) {
        const uint32_t m = G[f + j], val = G[f + L + j];
        if (m == 0xFFFFFFFFu) o << "  " << lim(j) << " = " << hex(val) << ";\n";
        else if (m) o << "  " << lim(j) << " = (" << lim(j) << " & " << hex(~m) << ") | " << hex(val) << ";\n";
      }
    }
    o << "  }\n";
    coord_var[c] = out;
  }

  std::string v(uint32_t id, uint32_t j) const {
    if (j >= Lw(P.vwidth[id])) return "0u";
    return "v" + std::to_string(id) + "_" + std::to_string(j);
  }
  static std::string hex(uint32_t x) {
    char b[16];
    snprintf(b, sizeof b, "0x%08xu", x);
    return b;
  }
  static uint32_t topmask(uint32_t w) { return (w & 31) ? ((1u << (w & 31)) - 1u) : 0xFFFFFFFFu; }
  // lo + x for every 0 <= x <= (maxadd << sh), over L limbs: the number k of low limbs that can
  // differ from lo's.  lo <= lo + x <= lo + max and, when that does not wrap, lo and lo + max agree
  // on every limb >= k, so lo + x does too: those limbs are literals and the carry chain stops at
  // limb k - 1.  L when the sum can wrap.
  static uint32_t reach_limbs(const uint32_t* lo, uint32_t L, uint64_t maxadd, uint32_t sh) {
    std::vector<uint32_t> add(L + 3, 0u);
    const uint32_t q = sh / 32, r = sh % 32;
    const unsigned __int128 x = (unsigned __int128)maxadd << r;
    for (uint32_t t = 0; t < 3 && q + t < L + 3; t++) add[q + t] = (uint32_t)(x >> (32 * t));
    for (uint32_t j = L; j < L + 3; j++)
      if (add[j]) return L;  // the addend alone reaches past the value
    uint64_t cy = 0;
    uint32_t k = 0;
    for (uint32_t j = 0; j < L; j++) {
      const uint64_t t = (uint64_t)lo[j] + add[j] + cy;
      if ((uint32_t)t != lo[j]) k = j + 1;
      cy = t >> 32;
    }
    return cy ? L : k;
  }

  // Bits [p, p+need) of value `id` (width w) as an expression in the low bits, zero above
  // `need` (bits at or above a value's width are zero by invariant).  Looks through CONCAT /
  // ZEXT / EXTRACT definitions down to their operands and literals, collecting pieces
  // (source value, source bit, length, destination bit); pieces that continue each other in
  // the same source merge, so a calldata word re-assembled from 32 byte-Extracts of one
  // 256-bit AUX word is one funnel shift per limb (v_alignbit_b32), and literal pieces fold
  // into one immediate.
  struct Piece {
    uint32_t id, w, p, n, sh;  // id == MG_NONE: literal bits `p` (already shifted to 0)
  };
  void collect(uint32_t id, uint32_t w, uint32_t p, uint32_t need, uint32_t sh, int depth,
               std::vector<Piece>& out) const {
    if (p >= w || need == 0) return;
    need = std::min(need, w - p);
    const Instr* d = def_of(id);
    if (d && depth < 96) {
      if (d->op == K_CONCAT) {
        const uint32_t wb = d->p1, wa = w - wb;
        if (p >= wb) return collect(d->a, wa, p - wb, need, sh, depth + 1, out);
        const uint32_t nlo = std::min(need, wb - p);
        collect(d->b, wb, p, nlo, sh, depth + 1, out);
        if (need > nlo) collect(d->a, wa, 0, need - nlo, sh + nlo, depth + 1, out);
        return;
      }
      if (d->op == K_ZEXT) return collect(d->a, d->p1, p, need, sh, depth + 1, out);
      if (d->op == K_EXTRACT) return collect(d->a, d->p1, d->p0 + p, need, sh, depth + 1, out);
      if (const uint32_t* c = lit(id)) {
        const uint32_t q = p >> 5, r = p & 31, L = Lw(w);
        uint32_t x = c[q] >> r;
        if (r && q + 1 < L) x |= c[q + 1] << (32 - r);
        if (need < 32) x &= (1u << need) - 1u;
        out.push_back({MG_NONE, 0, x, need, sh});
        return;
      }
    }
    out.push_back({id, w, p, need, sh});
  }

  std::string bits(uint32_t id, uint32_t w, uint32_t p, int need = 32) const {
    std::vector<Piece> ps;
    collect(id, w, p, (uint32_t)std::max(need, 0), 0, 0, ps);
    std::vector<Piece> m;
    uint32_t litv = 0;
    for (const Piece& q : ps) {
      if (q.id == MG_NONE) {
        litv |= q.sh < 32 ? q.p << q.sh : 0u;
        continue;
      }
      if (!m.empty() && m.back().id == q.id && m.back().p + m.back().n == q.p && m.back().sh + m.back().n == q.sh) {
        m.back().n += q.n;
        continue;
      }
      m.push_back(q);
    }
    std::string e;
    for (const Piece& q : m) {
      const uint32_t qq = q.p >> 5, r = q.p & 31, L = Lw(q.w);
      std::string x;
      if (r == 0) x = v(q.id, qq);
      else if (qq + 1 < L && q.n > 32 - r)
        x = "__builtin_amdgcn_alignbit(" + v(q.id, qq + 1) + ", " + v(q.id, qq) + ", " + std::to_string(r) + ")";
      else x = "(" + v(q.id, qq) + " >> " + std::to_string(r) + ")";
      if (q.n < 32 && q.p + q.n < q.w) x = "(" + x + " & " + hex((1u << q.n) - 1u) + ")";
      if (q.sh) x = "(" + x + " << " + std::to_string(q.sh) + ")";
      e = e.empty() ? x : "(" + e + " | " + x + ")";
    }
    if (litv) e = e.empty() ? hex(litv) : "(" + e + " | " + hex(litv) + ")";
    return e.empty() ? "0u" : e;
  }

  // x <op> c / c <op> x with a literal c that fits in limb 0 (and, for signed
  // compares, is non-negative): only limb 0 is compared; the upper limbs enter
  // through one OR-reduction written identically everywhere so LLVM CSEs it
  // across all compares of the same value (e.g. every `i < calldatasize`).
  bool emit_small_literal_compare(const Instr& in, uint32_t d, uint32_t wa, uint32_t La, bool sgn) {
    if (La < 2 || wa <= 32) return false;
    const uint32_t* la = lit(in.a);
    const uint32_t* lb = lit(in.b);
    if ((la == nullptr) == (lb == nullptr)) return false;
    const uint32_t* c = la ? la : lb;
    for (uint32_t j = 1; j < La; j++)
      if (c[j]) return false;
    const uint32_t x = la ? in.b : in.a;  // the non-literal operand
    const bool lit_left = la != nullptr;
    std::string hz = "((0u";
    for (uint32_t j = 1; j < La; j++) hz += " | " + v(x, j);
    hz += ") == 0u)";
    const std::string c0 = hex(c[0]);
    const std::string neg = "((" + v(x, La - 1) + " >> " + std::to_string((wa - 1) & 31) + ") & 1u)";
    const bool strict = in.op == K_ULT || in.op == K_SLT;
    std::string e;
    if (!lit_left) {
      // x < c  |  x <= c
      e = "(" + hz + " && " + v(x, 0) + (strict ? " < " : " <= ") + c0 + ")";
      if (sgn) e = "(" + neg + " || " + e + ")";
    } else {
      // c < x  = !(x <= c)  |  c <= x = !(x < c)
      e = "!(" + hz + " && " + v(x, 0) + (strict ? " <= " : " < ") + c0 + ")";
      if (sgn) e = "(!" + neg + " && " + e + ")";
    }
    o << "  " << v(d, 0) << " = (uint32_t)(" << e << ");\n";
    return true;
  }

  void mask_top(uint32_t id) {
    const uint32_t w = P.vwidth[id];
    if (w & 31) o << "  " << v(id, Lw(w) - 1) << " &= " << hex(topmask(w)) << ";\n";
  }

  std::string w8(uint32_t id) const {
    std::string s = "{{";
    for (uint32_t j = 0; j < 8; j++) s += (j ? "," : "") + v(id, j);
    return s + "}}";
  }

  void emit(const Instr& in, bool search, bool eval_watch) {
    const uint32_t d = in.dst, W = in.wd, L = Lw(W);
    switch (in.op) {
      case K_CONST:
        for (uint32_t j = 0; j < L; j++) o << "  " << v(d, j) << " = " << hex(P.consts[in.p0 + j]) << ";\n";
        break;
      case K_COORD:
        if (search) {
          gen_value(in.p0, "v" + std::to_string(d));
        } else {
          for (uint32_t j = 0; j < L; j++) {
            if (!P.watch_words || walk_watch()) {
              // no watch rows: one pointer walks the SoA rows (the loads come in row order, at the
              // loop's top level), each load a 64-bit add of a small multiple of n to the previous
              // address.  With soa[K * n + i] LLVM hoists every row's K * n out of the candidate
              // loop into SGPR pairs and spills them to VGPR lanes (C4: ~970 v_readlane +
              // ~970 v_writelane per candidate).  A program with watch rows keeps the indexed form
              // (its per-store branches compile too slowly around the walking pointer's barriers)
              const int64_t step = (int64_t)(in.p1 + j) - (int64_t)soa_row;
              if (step && tiled) o << "  sp_ += " << step * 64 << "ll; __asm__ volatile(\"\" : \"+v\"(sp_));\n";
              else if (step) o << "  sp_ += (long long)" << step << " * (long long)n; __asm__ volatile(\"\" : \"+v\"(sp_));\n";
              o << "  " << v(d, j) << " = *sp_;  // soa row " << (in.p1 + j) << "\n";
              soa_row = in.p1 + j;
            } else {
              if (tiled)
                o << "  " << v(d, j) << " = soa[((i >> 6) * " << P.coord_words << "ull + " << (in.p1 + j) << "ull) * 64ull + (i & 63ull)];\n";
              else
                o << "  " << v(d, j) << " = soa[(uint64_t)" << (in.p1 + j) << "u * n + i];\n";
            }
          }
        }
        break;
      case K_ADD:
      case K_SUB: {
        const bool sub = in.op == K_SUB;
        // carry / borrow chain: one v_add_co / v_addc_co (v_sub_co / v_subb_co) per limb
        o << "  { uint32_t c = 0u;";
        for (uint32_t j = 0; j < L; j++)
          o << " " << v(d, j) << " = " << (sub ? "mg_subc(" : "mg_addc(") << v(in.a, j) << ", "
            << v(in.b, j) << ", c, &c);";
        o << " (void)c; }\n";
        mask_top(d);
        break;
      }
      case K_NEG: {
        o << "  { uint32_t c = 0u;";
        for (uint32_t j = 0; j < L; j++) o << " " << v(d, j) << " = mg_subc(0u, " << v(in.a, j) << ", c, &c);";
        o << " (void)c; }\n";
        mask_top(d);
        break;
      }
      case K_AND: case K_OR: case K_XOR: {
        const char* op = in.op == K_AND ? " & " : in.op == K_OR ? " | " : " ^ ";
        for (uint32_t j = 0; j < L; j++) o << "  " << v(d, j) << " = " << v(in.a, j) << op << v(in.b, j) << ";\n";
        break;
      }
      case K_NOT:
        for (uint32_t j = 0; j < L; j++) o << "  " << v(d, j) << " = ~" << v(in.a, j) << ";\n";
        mask_top(d);
        break;
      case K_ITE:
        for (uint32_t j = 0; j < L; j++)
          o << "  " << v(d, j) << " = " << v(in.a, 0) << " ? " << v(in.b, j) << " : " << v(in.c, j) << ";\n";
        break;
      case K_EQ: {
        const uint32_t La = Lw(in.p1);
        o << "  " << v(d, 0) << " = (0u";
        for (uint32_t j = 0; j < La; j++) o << " | (" << v(in.a, j) << " ^ " << v(in.b, j) << ")";
        o << ") == 0u;\n";
        break;
      }
      case K_ULT: case K_ULE: case K_SLT: case K_SLE: {
        const uint32_t wa = in.p1, La = Lw(wa);
        const bool sgn = in.op == K_SLT || in.op == K_SLE;
        if (emit_small_literal_compare(in, d, wa, La, sgn)) break;
        const std::string flip = sgn ? hex(1u << ((wa - 1) & 31)) : "0u";
        o << "  { uint32_t br = 0u, nz = 0u;";
        for (uint32_t j = 0; j < La; j++) {
          std::string x = v(in.a, j), y = v(in.b, j);
          if (j == La - 1 && sgn) {
            x = "(" + x + " ^ " + flip + ")";
            y = "(" + y + " ^ " + flip + ")";
          }
          o << " nz |= mg_subc(" << x << ", " << y << ", br, &br);";
        }
        if (in.op == K_ULT || in.op == K_SLT)
          o << " " << v(d, 0) << " = (uint32_t)br; (void)nz; }\n";
        else
          o << " " << v(d, 0) << " = (uint32_t)(br != 0 || nz == 0); }\n";
        break;
      }
      case K_CONCAT:
      case K_EXTRACT:
        // through the value's own definition: bits() merges the pieces across both operands
        for (uint32_t j = 0; j < L; j++) o << "  " << v(d, j) << " = " << bits(d, W, 32 * j) << ";\n";
        break;
      case K_ZEXT: {
        const uint32_t La = Lw(in.p1);
        for (uint32_t j = 0; j < L; j++) o << "  " << v(d, j) << " = " << (j < La ? v(in.a, j) : "0u") << ";\n";
        break;
      }
      case K_SEXT: {
        const uint32_t wa = in.p1, La = Lw(wa);
        const uint32_t tm = topmask(wa);
        o << "  { const uint32_t f = ((" << v(in.a, La - 1) << " >> " << ((wa - 1) & 31) << ") & 1u) ? 0xFFFFFFFFu : 0u;";
        for (uint32_t j = 0; j < L; j++) {
          if (j < La - 1) o << " " << v(d, j) << " = " << v(in.a, j) << ";";
          else if (j == La - 1)
            o << " " << v(d, j) << " = (" << v(in.a, j) << " & " << hex(tm) << ") | (f & " << hex(~tm) << ");";
          else o << " " << v(d, j) << " = f;";
        }
        o << " }\n";
        mask_top(d);
        break;
      }
      case K_MUL: case K_UDIV: case K_UREM: case K_SDIV: case K_SREM: case K_SMOD:
      case K_SHL: case K_LSHR: case K_ASHR: case K_EXP: {
        const char* fn = nullptr;
        switch (in.op) {
          case K_MUL: fn = "mul8w"; break;
          case K_UDIV: fn = "bv_udiv"; break;
          case K_UREM: fn = "bv_urem"; break;
          case K_SDIV: fn = "bv_sdiv"; break;
          case K_SREM: fn = "bv_srem"; break;
          case K_SMOD: fn = "bv_smod"; break;
          case K_SHL: fn = "bv_shl"; break;
          case K_LSHR: fn = "bv_lshr"; break;
          case K_ASHR: fn = "bv_ashr"; break;
          default: fn = "bv_exp"; break;
        }
        o << "  { const W8 x = " << w8(in.a) << ", y = " << w8(in.b) << "; const W8 r = " << fn << "(x, y, " << W
          << "u);";
        for (uint32_t j = 0; j < L; j++) o << " " << v(d, j) << " = r.w[" << j << "];";
        o << " }\n";
        break;
      }
      case K_UMUL_NOOVF: {
        const uint32_t wa = in.p1;
        o << "  { const W8 x = " << w8(in.a) << ", y = " << w8(in.b) << "; " << v(d, 0) << " = umul_noovf8(x, y, "
          << wa << "u); }\n";
        break;
      }
      case K_LOOKUP: {
        const uint32_t Lk = Lw(in.b), n = in.c;
        for (uint32_t j = 0; j < L; j++) o << "  " << v(d, j) << " = " << v(in.p0, j) << ";\n";
        // first match wins: apply the priors from last to first.  MYTHGPU_JIT_LOOKUP_GATE=1:
        // limb 0 decides for the whole wave first (one compare and a ballot) and the full
        // compare + select runs only when some lane's limb 0 matches — measured no faster on
        // C1-C4 (their keys coincide in some lane of most waves), so off by default.
        static const bool gate = [] {
          const char* g = getenv("MYTHGPU_JIT_LOOKUP_GATE");
          return g && g[0] == '1';
        }();
        for (int32_t p = (int32_t)n - 1; p >= 0; p--) {
          const uint32_t kv = P.vaux[in.p1 + 2 * p], vv = P.vaux[in.p1 + 2 * p + 1];
          if (gate && Lk > 1) {
            o << "  { const bool h0 = " << v(in.a, 0) << " == " << v(kv, 0) << ";";
            o << " if (__builtin_amdgcn_ballot_w64(h0)) { const bool h = h0 && (0u";
            for (uint32_t j = 1; j < Lk; j++) o << " | (" << v(in.a, j) << " ^ " << v(kv, j) << ")";
            o << ") == 0u;";
            for (uint32_t j = 0; j < L; j++) o << " " << v(d, j) << " = h ? " << v(vv, j) << " : " << v(d, j) << ";";
            o << " } }\n";
            continue;
          }
          o << "  { const bool h = (0u";
          for (uint32_t j = 0; j < Lk; j++) o << " | (" << v(in.a, j) << " ^ " << v(kv, j) << ")";
          o << ") == 0u;";
          for (uint32_t j = 0; j < L; j++) o << " " << v(d, j) << " = h ? " << v(vv, j) << " : " << v(d, j) << ";";
          o << " }\n";
        }
        break;
      }
      case K_KECCAK: {
        if (in.a == MG_NONE) {
          static const uint32_t e[8] = {0x5d85a470u, 0x7bfad804u, 0xca82273bu, 0xe500b653u,
                                        0xdcc703c0u, 0x927e7db2u, 0x86f7233cu, 0xc5d24601u};
          for (uint32_t j = 0; j < 8; j++) o << "  " << v(d, j) << " = " << hex(e[j]) << ";\n";
        } else {
          const uint32_t La = Lw(P.vwidth[in.a]);
          o << "  { uint32_t in_[" << La << "] = {";
          for (uint32_t j = 0; j < La; j++) o << (j ? "," : "") << v(in.a, j);
          o << "}; uint32_t out_[8]; keccak_value<" << La << ", " << in.p0 << ">(in_, out_);";
          for (uint32_t j = 0; j < 8; j++) o << " " << v(d, j) << " = out_[" << j << "];";
          o << " }\n";
        }
        break;
      }
      case K_ASSERT:
        o << "  verdict &= " << v(in.a, 0) << ";\n";
        if (search) o << "  if (early && __ballot(verdict != 0u) == 0ull) goto mg_next;\n";
        break;
      case K_WATCH:
        if (eval_watch) {
          for (uint32_t j = 0; j < L; j++) {
            if (walk_watch()) {
              // the watch rows through a walking pointer too: indexed stores had LLVM hoist every
              // row's K * n into SGPR pairs and spill them to VGPR lanes (C4: 974 v_readlane +
              // 972 v_writelane)
              const int64_t step = (int64_t)(in.p0 + j) - (int64_t)watch_row;
              // n through an opaque copy: step * n is then computed at the store, not hoisted out of
              // the candidate loop into one SGPR pair per row (54 v_writelane spills on C4)
              if (step)
                o << "  { uint64_t n_ = n; __asm__ volatile(\"\" : \"+s\"(n_)); wp_ += (long long)" << step
                  << " * (long long)n_; __asm__ volatile(\"\" : \"+v\"(wp_)); }\n";
              o << "  if (watch) *wp_ = " << v(in.a, j) << ";\n";
              watch_row = in.p0 + j;
            } else {
              o << "  if (watch) watch[(uint64_t)" << (in.p0 + j) << "u * n + i] = " << v(in.a, j) << ";\n";
            }
          }
        }
        break;
      case K_COPY:
        for (uint32_t j = 0; j < L; j++) o << "  " << v(d, j) << " = " << v(in.a, j) << ";\n";
        break;
      default:
        break;
    }
  }

  void decls() {
    // declare every limb of every value the code defines or reads, up front (gotos may jump over
    // the body).  Only those: the value ids are the unspecialised program's, and declaring all of
    // them (C2: 4,385 limbs for 287 used) was a large share of the compiler's front-end time.
    std::vector<char> used(P.vwidth.size(), 0);
    auto mark = [&](uint32_t id) {
      if (id != MG_NONE && id < used.size()) used[id] = 1;
    };
    for (const Instr& in : P.vcode) {
      mark(in.dst);
      if (in.op == K_CONST || in.op == K_COORD) continue;
      mark(in.a);
      if (in.op == K_LOOKUP) {
        mark(in.p0);
        for (uint32_t q = 0; q < 2 * in.c; q++) mark(P.vaux[in.p1 + q]);
        continue;
      }
      mark(in.b);
      mark(in.c);
    }
    size_t n = 0;
    for (uint32_t id = 0; id < P.vwidth.size(); id++) {
      if (!used[id]) continue;
      for (uint32_t j = 0; j < Lw(P.vwidth[id]); j++) {
        o << (n % 16 == 0 ? "  uint32_t " : ", ") << v(id, j);
        if (n % 16 == 15) o << ";\n";
        n++;
      }
    }
    if (n % 16) o << ";\n";
  }

  // P is specialised (program.cpp specialize_program): decided compares are literals,
  // aliases are renamed away and dead instructions are gone
  uint32_t soa_row = 0;  // eval kernel without watch rows: the SoA row sp_ points at
  uint32_t watch_row = 0;  // the watch row wp_ points at
  // MYTHGPU_JIT_WATCH_WALK=1: eval kernels with watch rows walk their SoA and watch rows with
  // pointers too.  It removes the K * n spills (C4: 974 v_readlane + 972 v_writelane -> 18 + 18, static
  // VALU 5,059 -> 3,114) but LLVM takes far longer over the per-store branches: a VMTests replay kernel
  // (TestNameRegistrator, 8 watch words) went from 184 s to past 300 s on this host.  So it is opt-in;
  // the spill-free watch-row kernel is the first tier's (jit_asm.cpp: its own register allocation)
  static bool walk_watch() {
    static const bool walk = [] {
      const char* g = getenv("MYTHGPU_JIT_WATCH_WALK");
      return g && g[0] == '1';
    }();
    return walk;
  }
  // MG_JIT_SOA_TILED: row r of candidate i at ((i / 64) * coord_words + r) * 64 + i % 64 (a group's
  // rows contiguous; jit_asm.cpp "Tiled SoA"): the walking pointer steps 64 words per row
  bool tiled = false;

  void body(bool search) {
    coord_var.clear();  // generated-coordinate names are per kernel
    // MYTHGPU_JIT_GEN_ONLY=1 (diagnostic, search kernels): only the candidate generator, its
    // limbs folded into the verdict so none is dead — the generator's share of the kernel time
    static const bool gen_only = [] {
      const char* g = getenv("MYTHGPU_JIT_GEN_ONLY");
      return g && g[0] == '1';
    }();
    if (search && gen_only) {
      o << "  { uint32_t fold_ = 0u;\n";
      for (const Instr& in : P.vcode) {
        if (in.op != K_COORD || ((*specs)[in.p0].kind & 0xFFu) == MG_GEN_LAZY) continue;
        // MYTHGPU_JIT_GEN_KIND=<k>: only the coordinates of generator kind k (mythgpu.h mg_gen_kind)
        if (const char* gk = getenv("MYTHGPU_JIT_GEN_KIND"))
          if (((*specs)[in.p0].kind & 0xFFu) != (uint32_t)atoi(gk)) continue;
        emit(in, true, false);
        for (uint32_t j = 0; j < Lw(in.wd); j++) o << "  fold_ ^= " << v(in.dst, j) << ";\n";
      }
      o << "  verdict &= (uint32_t)(fold_ == 0x9E3779B9u); }\n";
      return;
    }
    soa_row = 0;  // eval: sp_ = soa + i addresses row 0
    watch_row = 0;
    for (const Instr& in : P.vcode) emit(in, search, !search);
  }
};

}  // namespace

std::string jit_source(const Lowered& P, const std::vector<GenSpec>* specs, const std::vector<uint32_t>* gconsts,
                       uint32_t kernels) {
  const bool want_search = kernels & JIT_SEARCH, want_eval = kernels & JIT_EVAL, want_gen = kernels & JIT_GEN;
  Gen g(P, specs, gconsts);
  g.tiled = (kernels & JIT_EVAL_TILED) != 0;
  g.plan_dict_lds();
  g.plan_dict_gv();
  g.plan_ws_slots();
  auto& o = g.o;
  // hipRTC compiles this with -nogpuinc -nogpulib: its own runtime header still supplies
  // __ballot/atomicMin/..., but no device library is linked (the kernels read work-item
  // ids through the clang builtins, so nothing references one) and clang's HIP wrapper
  // headers are skipped, which together take ~1/3 off hipRTC's fixed cost.
  o << "typedef unsigned int uint32_t;\ntypedef int int32_t;\ntypedef unsigned long long uint64_t;\n"
       "typedef unsigned char uint8_t;\n";
  o << kPrelude << "\nusing namespace mg;\n";
  o << "typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));\n"
       "typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));\n";
  g.emit_dict_gv_table();
  // 256-lane blocks; optional occupancy target (min waves per SIMD) for the search kernel
  std::string lb = "__attribute__((amdgpu_flat_work_group_size(1, 256)))";
  if (const char* wv = getenv("MYTHGPU_JIT_WAVES"))
    if (atoi(wv) > 0) lb += " __attribute__((amdgpu_waves_per_eu(" + std::to_string(atoi(wv)) + ")))";
  if (want_search) {
  // search kernel
  o << "extern \"C\" __global__ void " << lb << " mgj_search(const uint32_t* __restrict__ gconsts, "
       "uint64_t start, uint64_t count, uint64_t sk, uint64_t sg, unsigned long long* hit, uint32_t flags, uint32_t nblk) {\n"
       "  // work-item ids from the builtins (no device library: hipRTC links none, -nogpulib)\n"
       "  const uint32_t tid = __builtin_amdgcn_workitem_id_x(), bid = __builtin_amdgcn_workgroup_id_x();\n"
       "  const bool early = (flags & 1u) != 0u;\n"
       "  const uint32_t lane = tid & 63u;\n"
       "  const uint64_t LK = fmix64((uint64_t)lane ^ sk);  // lane half of the lane key (GEN3)\n"
       ;
  g.emit_dict_prologue();
  o << "  __shared__ unsigned long long mg_blk[2];  // the block's first hit and hit count\n"
       "  __shared__ uint32_t mg_blk_n;  // waves of the block that have added theirs\n"
       "  if (tid == 0u) { mg_blk[0] = ~0ull; mg_blk[1] = 0ull; mg_blk_n = 0u; }\n"
       "  __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"workgroup\");\n"
       "  __builtin_amdgcn_s_barrier();\n"
       "  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"workgroup\");\n";
  o << "  // one aligned group of 64 candidate indices per wave (GEN3 group key, mythgpu.h)\n"
       "  const uint64_t a0 = start & ~63ull, end = start + count;\n"
       "  const uint64_t ngroups = (end - a0 + 63ull) >> 6;\n"
       "  const uint64_t gstride = (uint64_t)nblk * 4u;  // 4 waves per 256-lane block\n"
       "  uint64_t wave_best = ~0ull, wave_hits = 0;  // per-wave, wave-uniform\n"
       "  // the wave's index in its block through readfirstlane: the group loop, its bookkeeping and\n"
       "  // wave_best / wave_hits are then scalar (from tid >> 6 they looked per-lane: a divergent loop\n"
       "  // with 64-bit VALU counters and exec-mask exits)\n"
       "  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);\n";
  g.emit_ws_salt();
  o << "  // this wave sweeps groups g0, g0 + gstride, ...: nk of them, counted in 32 bits (the engine\n"
       "  // launches at most 2^52 candidates); the call's partial first / last group, as iteration numbers\n"
       "  const uint64_t g0 = (uint64_t)bid * 4u + wv;\n"
       "  // (32-bit division when the operands fit: a 64-bit one is a long call per wave)\n"
       "  const uint64_t gleft = g0 < ngroups ? ngroups - 1u - g0 : 0u;\n"
       "  const uint32_t nk = g0 >= ngroups ? 0u : ((gleft >> 32) == 0u && (gstride >> 32) == 0u)\n"
       "      ? (uint32_t)gleft / (uint32_t)gstride + 1u : (uint32_t)(gleft / gstride + 1u);\n"
       "  const uint32_t kpf = (g0 == 0u && (start & 63u)) ? 0u : 0xFFFFFFFFu;\n"
       "  const uint32_t kpl = ((end & 63u) && nk && g0 + (uint64_t)(nk - 1u) * gstride == ngroups - 1u) ? nk - 1u : 0xFFFFFFFFu;\n"
       "  uint64_t gbase = a0 + (g0 << 6);\n";
  g.plan_prefetch();
  if (!g.pf.empty()) {
    o << "  uint64_t Gn = fmix64((gbase >> 6) ^ sg);  // the key of the wave's next group (prefetch)\n";
    g.emit_prefetch_decls();
    g.emit_prefetch("Gn");
  }
  o << "  for (uint32_t kk = 0u; kk < nk; kk++, gbase += gstride << 6) {\n"
       "  uint64_t cu = ~0ull;  // the hit word as this group starts (early exit only)\n"
       "  if (early) {\n"
       "    // system scope when peers on other GPUs lower this word (MG_SEARCH_SYSTEM_SCOPE, mg_init)\n"
       "    const unsigned long long cur = (flags & 2u) ? __hip_atomic_load(hit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)\n"
       "                                               : __hip_atomic_load(hit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);\n"
       "    cu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(cur >> 32)) << 32) | "
       "(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)cur);\n"
       "    if (gbase >= cu) break;\n"
       "  }\n"
       "  // a group wholly inside [start, end) (every group of a call but its first and last) needs no\n"
       "  // per-lane bounds\n"
       "  const bool full = kk != kpf && kk != kpl;\n";
  if (g.pf.empty()) {
    g.emit_group_keys("kk", "g0 + (uint64_t)kk * gstride", "gstride");
  } else {
    o << "  const uint64_t G = Gn;\n";
    g.emit_prefetch_take();
    o << "  Gn = fmix64(((gbase >> 6) + gstride) ^ sg);\n";
    g.emit_prefetch("Gn");
  }
  o << "  GKeys ky;\n"
       "  { const uint64_t K = G ^ LK;\n"
       "    ky.klo = (uint32_t)K; ky.khi = (uint32_t)(K >> 32); ky.kf = ky.klo ^ (ky.klo >> 16); ky.glo = (uint32_t)G;\n"
       "    ky.ghi = (uint32_t)(G >> 32); }\n"
       "  uint32_t verdict = 1u;\n";
  g.decls();
  g.pf_active = true;
  g.body(true);
  g.pf_active = false;
  o << "  mg_next:\n"
       "  { unsigned long long m = __ballot(verdict != 0u);\n"
       "    if (!full) { const uint64_t idx = gbase + lane; m &= __ballot(idx >= start && idx < end); }\n"
       "    if (m) {\n"
       "      const uint64_t first = gbase + (uint64_t)(__ffsll((long long)m) - 1);\n"
       "      wave_hits += (uint64_t)__popcll(m);\n"
       "      if (first < wave_best) {\n"
       "        wave_best = first;\n"
       "        // publish at once when waves stop early on it (and to the devices whose slices lie above\n"
       "        // this one's: the peer line at hit + 272, engine.hip kPeerWord); else once per wave at the end\n"
       "        // (a hit at or above the word read as the group started cannot lower it: no atomic)\n"
       "        if (early && lane == 0u && first < cu) {\n"
       "          atomicMin(hit, (unsigned long long)first);\n"
       "          const uint32_t np = (uint32_t)hit[272];\n"
       "          for (uint32_t q = 0u; q < np && q < 15u; q++)\n"
       "            __hip_atomic_fetch_min((unsigned long long*)hit[273u + q], (unsigned long long)first, __ATOMIC_RELAXED,\n"
       "                                   __HIP_MEMORY_SCOPE_SYSTEM);\n"
       "        }\n"
       "      }\n"
       "    } }\n"
       "  }\n"
       "  // the block's four waves combine in LDS and the last of them to finish publishes: the\n"
       "  // end-of-wave global atomics on one address from every wave serialised in the launch's tail;\n"
       "  // a first hit that cannot lower the current minimum is not published at all.  No barrier:\n"
       "  // issue arbitration favours a SIMD's oldest wave, so a block's waves finish staggered and\n"
       "  // the first ones would idle there until the last\n"
       "  if (lane == 0u) {\n"
       "    if (wave_best != ~0ull) __hip_atomic_fetch_min(&mg_blk[0], (unsigned long long)wave_best, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);\n"
       "    if (wave_hits) __hip_atomic_fetch_add(&mg_blk[1], (unsigned long long)wave_hits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);\n"
       "    if (__hip_atomic_fetch_add(&mg_blk_n, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) == 3u) {\n"
       "      const unsigned long long bb = __hip_atomic_load(&mg_blk[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);\n"
       "      const unsigned long long bh = __hip_atomic_load(&mg_blk[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);\n"
       "      if (bb != ~0ull && bb < __hip_atomic_load(hit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(hit, bb);\n"
       "      if (bh) atomicAdd(hit + 16u * (1u + (bid & 15u)), bh);  // the block's count stripe (engine.hip kHitStripes)\n"
       "    }\n"
       "  }\n}\n\n";
  }
  if (want_gen) {
  // per-candidate verdicts of generated candidates [start, start + count) (parity tests)
  o << "extern \"C\" __global__ void " << lb << " mgj_gen(const uint32_t* __restrict__ gconsts, "
       "uint64_t start, uint64_t count, uint64_t sk, uint64_t sg, uint8_t* __restrict__ verdict_out, uint32_t nblk) {\n"
       "  const uint32_t tid = __builtin_amdgcn_workitem_id_x(), bid = __builtin_amdgcn_workgroup_id_x();\n"
       "  const bool early = false;\n"
       "  const uint32_t lane = tid & 63u;\n"
       "  const uint64_t LK = fmix64((uint64_t)lane ^ sk);  // lane half of the lane key (GEN3)\n";
  g.emit_dict_prologue();
  o << "  const uint64_t a0 = start & ~63ull, end = start + count;\n"
       "  const uint64_t ngroups = (end - a0 + 63ull) >> 6;\n"
       "  const uint64_t gstride = (uint64_t)nblk * 4u;\n"
       "  const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6);\n";
  g.emit_ws_salt();
  o << "  uint32_t kk = 0u;\n"
       "  for (uint64_t g = (uint64_t)bid * 4u + wv; g < ngroups; g += gstride, kk++) {\n"
       "  const uint64_t gbase = a0 + (g << 6);\n"
       "  const uint64_t idx = gbase + lane;\n"
       "  const bool active = idx >= start && idx < end;\n";
  g.emit_group_keys("kk", "g", "gstride");
  o << "  GKeys ky;\n"
       "  { const uint64_t K = G ^ LK;\n"
       "    ky.klo = (uint32_t)K; ky.khi = (uint32_t)(K >> 32); ky.kf = ky.klo ^ (ky.klo >> 16); ky.glo = (uint32_t)G;\n"
       "    ky.ghi = (uint32_t)(G >> 32); }\n"
       "  uint32_t verdict = 1u;\n";
  g.decls();
  g.body(true);
  o << "  mg_next:\n"
       "  if (active) verdict_out[idx - start] = (uint8_t)verdict;\n"
       "  }\n}\n\n";
  }
  if (want_eval) {
  // eval kernel (explicit SoA coordinates, verdicts, optional watch rows).  GU32: a
  // global-address-space word, so the walking row pointer stays global_load (a generic pointer
  // through the asm barrier would become flat); declared here, so search kernels' sources (and
  // the SHAs their profiles are matched by) do not change
  o << "typedef uint32_t __attribute__((address_space(1))) GU32;\n";
  o << "extern \"C\" __global__ void " << lb << " mgj_eval(const uint32_t* __restrict__ soa, uint64_t n, "
       "uint8_t* __restrict__ verdict_out, uint32_t* __restrict__ watch, uint32_t nblk) {\n"
       "  const uint64_t stride = (uint64_t)nblk * 256u;\n"
       "  for (uint64_t i = (uint64_t)__builtin_amdgcn_workgroup_id_x() * 256u + __builtin_amdgcn_workitem_id_x(); i < n; i += stride) {\n"
       "  uint32_t verdict = 1u;\n"
       << (g.tiled ? "  const GU32* sp_ = (const GU32*)((uint64_t)soa + (((i >> 6) * " + std::to_string(P.coord_words) +
                       "ull * 64ull) + (i & 63ull)) * 4ull);  // tiled SoA\n"
                 : std::string("  const GU32* sp_ = (const GU32*)((uint64_t)soa + i * 4ull);\n"));
  if (P.watch_words && Gen::walk_watch()) o << "  GU32* wp_ = (GU32*)((uint64_t)watch + i * 4ull);\n";
  g.decls();
  g.body(false);
  o << "  verdict_out[i] = (uint8_t)verdict;\n  }\n}\n";
  }
  return o.str();
}

// ---------------------------------------------------------------------------
// hipRTC, loaded at run time (no link-time dependency of libmythgpu.so on it)
// ---------------------------------------------------------------------------
namespace {
typedef int (*pCreate)(void**, const char*, const char*, int, const char**, const char**);
typedef int (*pCompile)(void*, int, const char**);
typedef int (*pSize)(void*, size_t*);
typedef int (*pGet)(void*, char*);
typedef int (*pDestroy)(void**);
struct Rtc {
  void* h = nullptr;
  pCreate create = nullptr;
  pCompile compile = nullptr;
  pSize log_size = nullptr, code_size = nullptr;
  pGet log = nullptr, code = nullptr;
  pDestroy destroy = nullptr;
  bool ok = false;
};
Rtc& rtc() {
  static Rtc r;
  if (r.h) return r;
  // fallback compiler (MYTHGPU_JIT_COMPILER=hiprtc or no comgr): the image's hipRTC by absolute
  // path; no dlmopen namespace (see comgr()).
  const char* names[] = {"/opt/rocm/lib/libhiprtc.so.7", "libhiprtc.so.7", "libhiprtc.so"};
  for (const char* n : names) {
    if (r.h) break;
    r.h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
  }
  if (!r.h) return r;
  r.create = (pCreate)dlsym(r.h, "hiprtcCreateProgram");
  r.compile = (pCompile)dlsym(r.h, "hiprtcCompileProgram");
  r.log_size = (pSize)dlsym(r.h, "hiprtcGetProgramLogSize");
  r.log = (pGet)dlsym(r.h, "hiprtcGetProgramLog");
  r.code_size = (pSize)dlsym(r.h, "hiprtcGetCodeSize");
  r.code = (pGet)dlsym(r.h, "hiprtcGetCode");
  r.destroy = (pDestroy)dlsym(r.h, "hiprtcDestroyProgram");
  r.ok = r.create && r.compile && r.log_size && r.log && r.code_size && r.code && r.destroy;
  return r;
}

// ---------------------------------------------------------------------------
// comgr (the compiler library hipRTC itself drives), called directly: source -> LLVM
// bitcode -> relocatable -> code object, with no hipRTC runtime header to parse and no
// device libraries to link (the kernels call none).  About half of hipRTC's latency per
// query kernel on this image; hipRTC stays as the fallback (MYTHGPU_JIT_COMPILER=hiprtc).
// ---------------------------------------------------------------------------
struct Comgr {
  void* h = nullptr;
  decltype(&amd_comgr_create_data) create_data = nullptr;
  decltype(&amd_comgr_set_data) set_data = nullptr;
  decltype(&amd_comgr_set_data_name) set_data_name = nullptr;
  decltype(&amd_comgr_release_data) release_data = nullptr;
  decltype(&amd_comgr_get_data) get_data = nullptr;
  decltype(&amd_comgr_create_data_set) create_set = nullptr;
  decltype(&amd_comgr_destroy_data_set) destroy_set = nullptr;
  decltype(&amd_comgr_data_set_add) set_add = nullptr;
  decltype(&amd_comgr_action_data_count) data_count = nullptr;
  decltype(&amd_comgr_action_data_get_data) data_get = nullptr;
  decltype(&amd_comgr_create_action_info) create_info = nullptr;
  decltype(&amd_comgr_destroy_action_info) destroy_info = nullptr;
  decltype(&amd_comgr_action_info_set_language) set_language = nullptr;
  decltype(&amd_comgr_action_info_set_isa_name) set_isa = nullptr;
  decltype(&amd_comgr_action_info_set_option_list) set_options = nullptr;
  decltype(&amd_comgr_action_info_set_logging) set_logging = nullptr;
  decltype(&amd_comgr_do_action) do_action = nullptr;
  bool ok = false;
};

Comgr& comgr() {
  static Comgr c;
  static std::once_flag once;
  std::call_once(once, [] {
    // by absolute path: the image's comgr, not torch's bundled copy of the same soname.  Not in
    // a fresh link namespace (dlmopen): that loads a second libc whose malloc also moves the
    // program break, and heap corruption follows once the compile thread runs beside the
    // caller's allocations.
    c.h = dlopen("/opt/rocm/lib/libamd_comgr.so.3", RTLD_NOW | RTLD_LOCAL);
    if (!c.h) c.h = dlopen("libamd_comgr.so.3", RTLD_NOW | RTLD_LOCAL);
    if (!c.h) return;
#define MG_SYM(field, name) c.field = (decltype(c.field))dlsym(c.h, #name)
    MG_SYM(create_data, amd_comgr_create_data);
    MG_SYM(set_data, amd_comgr_set_data);
    MG_SYM(set_data_name, amd_comgr_set_data_name);
    MG_SYM(release_data, amd_comgr_release_data);
    MG_SYM(get_data, amd_comgr_get_data);
    MG_SYM(create_set, amd_comgr_create_data_set);
    MG_SYM(destroy_set, amd_comgr_destroy_data_set);
    MG_SYM(set_add, amd_comgr_data_set_add);
    MG_SYM(data_count, amd_comgr_action_data_count);
    MG_SYM(data_get, amd_comgr_action_data_get_data);
    MG_SYM(create_info, amd_comgr_create_action_info);
    MG_SYM(destroy_info, amd_comgr_destroy_action_info);
    MG_SYM(set_language, amd_comgr_action_info_set_language);
    MG_SYM(set_isa, amd_comgr_action_info_set_isa_name);
    MG_SYM(set_options, amd_comgr_action_info_set_option_list);
    MG_SYM(set_logging, amd_comgr_action_info_set_logging);
    MG_SYM(do_action, amd_comgr_do_action);
#undef MG_SYM
    c.ok = c.create_data && c.set_data && c.set_data_name && c.release_data && c.get_data && c.create_set &&
           c.destroy_set && c.set_add && c.data_count && c.data_get && c.create_info && c.destroy_info &&
           c.set_language && c.set_isa && c.set_options && c.set_logging && c.do_action;
  });
  return c;
}

// what hipRTC's runtime header would provide, reduced to what the JIT kernels use
const char* kComgrShim = R"MGJ(
#define __device__ __attribute__((device))
#define __host__ __attribute__((host))
#define __global__ __attribute__((global))
#define __shared__ __attribute__((shared))
#define __constant__ __attribute__((constant))
#define __forceinline__ inline __attribute__((always_inline))
__device__ inline unsigned long long __ballot(int p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ inline int __ffsll(unsigned long long x) { return x ? __builtin_ctzll(x) + 1 : 0; }
__device__ inline int __popcll(unsigned long long x) { return __builtin_popcountll(x); }
__device__ inline unsigned long long atomicMin(unsigned long long* p, unsigned long long v) {
  return __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned long long atomicAdd(unsigned long long* p, unsigned long long v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
)MGJ";

const std::vector<std::string>& extra_options() {
  // MYTHGPU_JIT_EXTRA: extra space-separated compiler options (tuning experiments)
  static std::vector<std::string> extra;
  static std::once_flag once;
  std::call_once(once, [] {
    // passes that find nothing to do in the emitted straight-line code (the SLP vectoriser; the
    // generic loop unroller — every loop of the prelude carries its own #pragma unroll): the code
    // objects are byte-identical without them (C2, C4, C5 search kernels; an eval kernel with MUL,
    // division and shifts) and a compile takes ~15 % less time.  MYTHGPU_JIT_FAST=0: run them
    const char* fast = getenv("MYTHGPU_JIT_FAST");
    if (!(fast && fast[0] == '0')) {
      extra.push_back("-fno-slp-vectorize");
      extra.push_back("-fno-unroll-loops");
    }
    if (const char* e = getenv("MYTHGPU_JIT_EXTRA")) {
      std::istringstream is(e);
      std::string t;
      while (is >> t) extra.push_back(t);
    }
    // -structurizecfg-skip-uniform-regions: no exec-mask structurisation of wave-uniform
    // regions (the MIXED alternatives and the early-exit jumps are SGPR branches), as the
    // engine itself is built.  A non-default LLVM option: on by default only while the
    // compiler runs in its own process (a compiler abort then costs one kernel, not the
    // caller; a wrong kernel is caught by z3's re-check of every GPU model).  Kernel time
    // with it, this round (profiles/r03_skip_uniform_sweep.jsonl): C1 -1.2 %, C2 -3.1 %,
    // C3 -4.7 %, C4 -5.4 %, C5 -1.2 %.  MYTHGPU_JIT_SKIP_UNIFORM=0 / =1 forces it off / on.
    const char* u = getenv("MYTHGPU_JIT_SKIP_UNIFORM");
    const char* iso = getenv("MYTHGPU_JIT_ISOLATE");
    const bool isolated = !(iso && iso[0] == '0');
    if (u ? u[0] == '1' : isolated) {
      extra.push_back("-mllvm");
      extra.push_back("-structurizecfg-skip-uniform-regions");
    }
  });
  return extra;
}

// MYTHGPU_JIT_OPT: optimisation level (default -O3)
std::string opt_level() { return std::string("-O") + (getenv("MYTHGPU_JIT_OPT") ? getenv("MYTHGPU_JIT_OPT") : "3"); }

int comgr_compile(const std::string& src, std::vector<char>& code, std::string& log) {
  Comgr& c = comgr();
  const std::string full = std::string(kComgrShim) + src;
  const std::string optlvl = opt_level();
  std::vector<const char*> opts = {optlvl.c_str(), "-std=c++17", "-nogpuinc", "-nogpulib", "-Wno-unused-variable",
                                   "-Wno-uninitialized", "-Wno-sometimes-uninitialized"};
  for (const auto& t : extra_options()) opts.push_back(t.c_str());
  amd_comgr_data_t src_d{0};
  amd_comgr_data_set_t in{0}, bc{0}, rel{0}, exe{0};
  amd_comgr_action_info_t ai{0};
  int rc = MG_E_HIP;
  auto collect_log = [&](amd_comgr_data_set_t set) {
    size_t n = 0;
    if (c.data_count(set, AMD_COMGR_DATA_KIND_LOG, &n) != AMD_COMGR_STATUS_SUCCESS) return;
    for (size_t i = 0; i < n; i++) {
      amd_comgr_data_t d;
      if (c.data_get(set, AMD_COMGR_DATA_KIND_LOG, i, &d) != AMD_COMGR_STATUS_SUCCESS) continue;
      size_t sz = 0;
      if (c.get_data(d, &sz, nullptr) == AMD_COMGR_STATUS_SUCCESS && sz > 1) {
        std::string t(sz, '\0');
        c.get_data(d, &sz, &t[0]);
        log += t;
      }
      c.release_data(d);
    }
  };
  do {
    if (c.create_data(AMD_COMGR_DATA_KIND_SOURCE, &src_d) || c.set_data(src_d, full.size(), full.data()) ||
        c.set_data_name(src_d, "mythgpu_jit.hip"))
      break;
    if (c.create_set(&in) || c.create_set(&bc) || c.create_set(&rel) || c.create_set(&exe) || c.set_add(in, src_d)) break;
    if (c.create_info(&ai) || c.set_language(ai, AMD_COMGR_LANGUAGE_HIP) ||
        c.set_isa(ai, "amdgcn-amd-amdhsa--gfx950") || c.set_options(ai, opts.data(), opts.size()) ||
        c.set_logging(ai, true))
      break;
    const auto t0 = std::chrono::steady_clock::now();
    if (c.do_action(AMD_COMGR_ACTION_COMPILE_SOURCE_TO_BC, ai, in, bc)) {
      collect_log(bc);
      break;
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (c.do_action(AMD_COMGR_ACTION_CODEGEN_BC_TO_RELOCATABLE, ai, bc, rel)) {
      collect_log(rel);
      break;
    }
    const auto t2 = std::chrono::steady_clock::now();
    if (c.do_action(AMD_COMGR_ACTION_LINK_RELOCATABLE_TO_EXECUTABLE, ai, rel, exe)) {
      collect_log(exe);
      break;
    }
    if (getenv("MYTHGPU_JIT_TIMING")) {
      const auto t3 = std::chrono::steady_clock::now();
      auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
      fprintf(stderr, "mythgpu jit: %zu bytes source, front+opt %.1f ms, codegen %.1f ms, link %.1f ms\n",
              full.size(), ms(t0, t1), ms(t1, t2), ms(t2, t3));
    }
    size_t n = 0;
    amd_comgr_data_t o;
    if (c.data_count(exe, AMD_COMGR_DATA_KIND_EXECUTABLE, &n) || n != 1 ||
        c.data_get(exe, AMD_COMGR_DATA_KIND_EXECUTABLE, 0, &o))
      break;
    size_t sz = 0;
    if (c.get_data(o, &sz, nullptr) == AMD_COMGR_STATUS_SUCCESS && sz) {
      code.resize(sz);
      if (c.get_data(o, &sz, code.data()) == AMD_COMGR_STATUS_SUCCESS) rc = MG_OK;
    }
    c.release_data(o);
  } while (false);
  if (ai.handle) c.destroy_info(ai);
  for (amd_comgr_data_set_t s : {in, bc, rel, exe})
    if (s.handle) c.destroy_set(s);
  if (src_d.handle) c.release_data(src_d);
  if (rc != MG_OK && log.empty()) log = "comgr compile failed";
  return rc;
}

// assembly (the first tier, jit_asm.cpp) -> relocatable -> code object
int comgr_assemble(const std::string& src, std::vector<char>& code, std::string& log) {
  Comgr& c = comgr();
  amd_comgr_data_t src_d{0};
  amd_comgr_data_set_t in{0}, rel{0}, exe{0};
  amd_comgr_action_info_t ai{0};
  int rc = MG_E_HIP;
  auto collect_log = [&](amd_comgr_data_set_t set) {
    size_t n = 0;
    if (c.data_count(set, AMD_COMGR_DATA_KIND_LOG, &n) != AMD_COMGR_STATUS_SUCCESS) return;
    for (size_t i = 0; i < n; i++) {
      amd_comgr_data_t d;
      if (c.data_get(set, AMD_COMGR_DATA_KIND_LOG, i, &d) != AMD_COMGR_STATUS_SUCCESS) continue;
      size_t sz = 0;
      if (c.get_data(d, &sz, nullptr) == AMD_COMGR_STATUS_SUCCESS && sz > 1) {
        std::string t(sz, '\0');
        c.get_data(d, &sz, &t[0]);
        log += t;
      }
      c.release_data(d);
    }
  };
  do {
    if (c.create_data(AMD_COMGR_DATA_KIND_SOURCE, &src_d) || c.set_data(src_d, src.size(), src.data()) ||
        c.set_data_name(src_d, "mythgpu_jit.s"))
      break;
    if (c.create_set(&in) || c.create_set(&rel) || c.create_set(&exe) || c.set_add(in, src_d)) break;
    if (c.create_info(&ai) || c.set_language(ai, AMD_COMGR_LANGUAGE_NONE) ||
        c.set_isa(ai, "amdgcn-amd-amdhsa--gfx950") || c.set_logging(ai, true))
      break;
    const auto t0 = std::chrono::steady_clock::now();
    if (c.do_action(AMD_COMGR_ACTION_ASSEMBLE_SOURCE_TO_RELOCATABLE, ai, in, rel)) {
      collect_log(rel);
      break;
    }
    const auto t1 = std::chrono::steady_clock::now();
    if (c.do_action(AMD_COMGR_ACTION_LINK_RELOCATABLE_TO_EXECUTABLE, ai, rel, exe)) {
      collect_log(exe);
      break;
    }
    if (getenv("MYTHGPU_JIT_TIMING")) {
      const auto t2 = std::chrono::steady_clock::now();
      auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
      fprintf(stderr, "mythgpu jit asm: %zu bytes, assemble %.2f ms, link %.2f ms\n", src.size(), ms(t0, t1), ms(t1, t2));
    }
    log.clear();  // the driver's notes about unused options
    size_t n = 0;
    amd_comgr_data_t o;
    if (c.data_count(exe, AMD_COMGR_DATA_KIND_EXECUTABLE, &n) || n != 1 ||
        c.data_get(exe, AMD_COMGR_DATA_KIND_EXECUTABLE, 0, &o))
      break;
    size_t sz = 0;
    if (c.get_data(o, &sz, nullptr) == AMD_COMGR_STATUS_SUCCESS && sz) {
      code.resize(sz);
      if (c.get_data(o, &sz, code.data()) == AMD_COMGR_STATUS_SUCCESS) rc = MG_OK;
    }
    c.release_data(o);
  } while (false);
  if (ai.handle) c.destroy_info(ai);
  for (amd_comgr_data_set_t s : {in, rel, exe})
    if (s.handle) c.destroy_set(s);
  if (src_d.handle) c.release_data(src_d);
  if (rc != MG_OK && log.empty()) log = "comgr assembly failed";
  return rc;
}

int hiprtc_compile(const std::string& src, std::vector<char>& code, std::string& log) {
  Rtc& r = rtc();
  if (!r.ok) {
    log = "hipRTC not available";
    return MG_E_UNSUPPORTED;
  }
  void* prog = nullptr;
  if (r.create(&prog, src.c_str(), "mythgpu_jit.hip", 0, nullptr, nullptr) != 0) {
    log = "hiprtcCreateProgram failed";
    return MG_E_HIP;
  }
  const std::string optlvl = opt_level();
  std::vector<const char*> opts = {"--offload-arch=gfx950", optlvl.c_str(), "-std=c++17", "-nogpuinc", "-nogpulib",
                                   "-Wno-unused-variable", "-Wno-uninitialized", "-Wno-sometimes-uninitialized"};
  for (const auto& t : extra_options()) opts.push_back(t.c_str());
  int rc = r.compile(prog, (int)opts.size(), opts.data());
  size_t ls = 0;
  r.log_size(prog, &ls);
  if (ls > 1) {
    log.resize(ls);
    r.log(prog, &log[0]);
  }
  if (rc != 0) {
    r.destroy(&prog);
    return MG_E_HIP;
  }
  size_t cs = 0;
  r.code_size(prog, &cs);
  code.resize(cs);
  r.code(prog, code.data());
  r.destroy(&prog);
  return MG_OK;
}
}  // namespace

// ---------------------------------------------------------------------------
// The compiler in its own process (mythgpu_jitd, jitd.cpp).  comgr is LLVM: an internal error
// is report_fatal_error -> abort(), which inside the caller would end the Mythril analysis with
// no z3 fallback.  So by default the engine never loads comgr itself: every compile is one
// request over a socketpair to a helper started with posix_spawn on first use.  If the helper
// dies (LLVM abort, a signal), the compile that was in flight fails, the engine marks the JIT
// unavailable and every later compile fails at once — searches stay on the interpreter (k_run)
// for the rest of the process; there is no restart.  MYTHGPU_JIT_ISOLATE=0 compiles in-process.
//
// Protocol (host byte order, both directions on one SOCK_STREAM socket):
//   request:  u64 env_len, env ("NAME=VALUE\0" for every AMD_COMGR_* / MYTHGPU_JIT* variable of
//             the caller at this moment), u64 src_len, src
//   response: i32 rc, u64 code_len, code, u64 log_len, log
// ---------------------------------------------------------------------------
namespace {

struct Helper {
  std::mutex mu;
  pid_t pid = -1;
  int fd = -1;
  bool dead = false;
  std::string why;
};

// three helper processes: [0] compiles (clang + LLVM), [1] and [2] assemble the first tier — an
// assembly request never queues behind a ~140 ms compile, nor behind the assembly of a search that
// has already ended (a cancelled request in flight runs to its end: C5's hard query waited 8.3 ms
// behind the easy query's, profiles/r05e_bench_c5.err)
constexpr int kHelpers = 3;
Helper& helper(int lane = 0) {
  static Helper* h[kHelpers] = {new Helper, new Helper, new Helper};  // leaked: usable from exit handlers
  return *h[lane < 0 || lane >= kHelpers ? 0 : lane];
}

bool send_all(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t k = send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

bool recv_all(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    ssize_t k = recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= (size_t)k;
  }
  return true;
}

std::string helper_path() {
  if (const char* p = getenv("MYTHGPU_JITD")) return p;
  Dl_info info;
  if (dladdr((void*)&helper, &info) && info.dli_fname) {
    std::string lib(info.dli_fname);
    const size_t slash = lib.rfind('/');
    return (slash == std::string::npos ? std::string(".") : lib.substr(0, slash)) + "/mythgpu_jitd";
  }
  return "mythgpu_jitd";
}

extern "C" char** environ;

// caller holds h.mu
bool helper_start(Helper& h) {
  int sv[2];
  if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0, sv) != 0) {
    h.why = "socketpair failed";
    return false;
  }
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_adddup2(&fa, sv[1], 0);  // dup2 clears CLOEXEC on the child's copy
  posix_spawn_file_actions_adddup2(&fa, sv[1], 1);
  const std::string path = helper_path();
  char* argv[] = {(char*)path.c_str(), nullptr};
  pid_t pid = -1;
  const int rc = posix_spawn(&pid, path.c_str(), &fa, nullptr, argv, environ);
  posix_spawn_file_actions_destroy(&fa);
  close(sv[1]);
  if (rc != 0) {
    close(sv[0]);
    h.why = "cannot start " + path + ": " + strerror(rc);
    return false;
  }
  h.pid = pid;
  h.fd = sv[0];
  return true;
}

// caller holds h.mu: the helper is gone; record how, reap it, never start another
void helper_lost(Helper& h) {
  int status = 0;
  std::string how = "JIT compiler process " + std::to_string(h.pid);
  if (h.fd >= 0) close(h.fd);
  h.fd = -1;
  if (h.pid > 0 && waitpid(h.pid, &status, 0) == h.pid) {
    if (WIFSIGNALED(status)) how += " killed by signal " + std::to_string(WTERMSIG(status));
    else if (WIFEXITED(status)) how += " exited with status " + std::to_string(WEXITSTATUS(status));
  } else {
    how += " lost";
  }
  h.pid = -1;
  h.dead = true;
  h.why = how + "; the JIT is off for the rest of this process (searches stay on the interpreter)";
  fprintf(stderr, "mythgpu: %s\n", h.why.c_str());
}

std::string env_snapshot() {
  std::string env;
  for (char** e = environ; e && *e; e++)
    if (!std::strncmp(*e, "AMD_COMGR_", 10) || !std::strncmp(*e, "MYTHGPU_JIT", 11)) {
      env += *e;
      env.push_back('\0');
    }
  return env;
}

int helper_compile_on(Helper& h, std::unique_lock<std::mutex>& g, const std::string& src, std::vector<char>& code,
                      std::string& log, bool& available);

// lane: -1 picks one (an assembly goes to whichever of its two helpers is free)
int helper_compile(const std::string& src, std::vector<char>& code, std::string& log, bool& available, int lane = -1) {
  const bool is_asm = src.compare(0, std::strlen(kAsmMarker), kAsmMarker) == 0;
  if (!is_asm) {
    std::unique_lock<std::mutex> g(helper(0).mu);
    return helper_compile_on(helper(0), g, src, code, log, available);
  }
  if (lane == 1 || lane == 2) {
    std::unique_lock<std::mutex> g(helper(lane).mu);
    return helper_compile_on(helper(lane), g, src, code, log, available);
  }
  for (int l = 1; l <= 2; l++) {
    std::unique_lock<std::mutex> g(helper(l).mu, std::try_to_lock);
    if (g.owns_lock() && !helper(l).dead) return helper_compile_on(helper(l), g, src, code, log, available);
  }
  std::unique_lock<std::mutex> g(helper(1).mu);  // both busy: wait for the first
  return helper_compile_on(helper(1), g, src, code, log, available);
}

// caller holds h.mu (g)
int helper_compile_on(Helper& h, std::unique_lock<std::mutex>& g, const std::string& src, std::vector<char>& code,
                      std::string& log, bool& available) {
  (void)g;
  available = true;
  if (h.dead) {
    log = h.why;
    return MG_E_UNSUPPORTED;
  }
  if (h.fd < 0 && !helper_start(h)) {
    available = false;  // no helper binary: the caller may compile in-process
    return MG_E_UNSUPPORTED;
  }
  const std::string env = env_snapshot();
  const uint64_t el = env.size(), sl = src.size();
  int32_t rc = MG_E_HIP;
  uint64_t cl = 0, ll = 0;
  bool ok = send_all(h.fd, &el, 8) && send_all(h.fd, env.data(), el) && send_all(h.fd, &sl, 8) &&
            send_all(h.fd, src.data(), sl) && recv_all(h.fd, &rc, 4) && recv_all(h.fd, &cl, 8);
  if (ok) {
    code.resize(cl);
    ok = recv_all(h.fd, code.data(), cl) && recv_all(h.fd, &ll, 8);
  }
  if (ok) {
    log.resize(ll);
    ok = recv_all(h.fd, &log[0], ll);
  }
  if (!ok) {
    helper_lost(h);
    code.clear();
    log = h.why;
    return MG_E_UNSUPPORTED;
  }
  return rc;
}

}  // namespace

void jit_helper_stop() {
  for (int lane = 0; lane < kHelpers; lane++) {
    Helper& h = helper(lane);
    std::lock_guard<std::mutex> g(h.mu);
    if (h.fd >= 0) {
      close(h.fd);  // the helper exits on end of input
      h.fd = -1;
    }
    if (h.pid > 0) {
      int status;
      (void)waitpid(h.pid, &status, 0);
      h.pid = -1;
    }
  }
}

int jit_helper_pid() {
  Helper& h = helper();
  std::lock_guard<std::mutex> g(h.mu);
  return h.dead ? -2 : (int)h.pid;
}

static bool isolated() {
  const char* v = getenv("MYTHGPU_JIT_ISOLATE");
  return !(v && v[0] == '0');
}

void jit_helper_warm(const std::string& asm_src) {
  const char* w = getenv("MYTHGPU_JIT_WARM");
  if (!isolated() || (w && w[0] == '0')) return;
  // the first tier's helper: started, and `asm_src` (a tiny kernel) assembled and linked through
  // it, so the process start-up, comgr's load and LLVM's AMDGPU target set-up are paid here and
  // not by the first query's first-tier compile (cold 11.9 ms against ~4.6 ms warm on the box,
  // profiles/r04h_bench.json)
  if (!asm_src.empty()) {
    for (int lane = 1; lane <= 2; lane++) {  // both assembly helpers
      std::vector<char> code;
      std::string log;
      bool available = true;
      (void)helper_compile(asm_src, code, log, available, lane);
    }
  }
  // the compiler's helper: started only (its first compile loads comgr)
  Helper& h = helper(0);
  std::lock_guard<std::mutex> g(h.mu);
  if (h.fd < 0 && !h.dead) (void)helper_start(h);
}

void jit_compiler_preload() {
  if (isolated()) return;  // the compiler lives in the helper process
  const char* which = getenv("MYTHGPU_JIT_COMPILER");
  if (!(which && std::strcmp(which, "hiprtc") == 0) && comgr().ok) return;
  (void)rtc();
}

// ---------------------------------------------------------------------------
// On-disk code-object cache, shared by every process of one user: a query shape compiled once
// (~0.15 s of comgr on the box) loads from disk in later Mythril runs (re-analysis, CI, one
// contract's several entry points).  comgr's own cache (AMD_COMGR_CACHE) already skips most of
// the compile of a known source (C2: 392 -> 15 ms on the host); this one also skips the helper
// process and comgr altogether (a hit costs one file read).  The key is everything that
// decides the code object: the source, the compiler-relevant environment (AMD_COMGR_* /
// MYTHGPU_JIT* bar the controls of the caches, the timing switch and the helper's path), the
// compiler choice and this library's build (HIP version, build time).  File <dir>/<h1><h2>.co
// = 24-B header (magic, key length, h1) + the ELF code object; written to a temporary name and
// renamed, so readers never see a partial file.  Any failure — no directory, a short or
// foreign file — is a miss and never an error.
//   MYTHGPU_JIT_DISK_CACHE=<dir>  cache directory (default ${XDG_CACHE_HOME:-$HOME/.cache}/mythgpu/jit)
//   MYTHGPU_JIT_DISK_CACHE=0      off
// ---------------------------------------------------------------------------
namespace {

constexpr uint64_t kCoMagic = 0x31304F43474D594Dull;  // "MYMGCO01"

std::string disk_cache_dir() {
  const char* d = getenv("MYTHGPU_JIT_DISK_CACHE");
  if (d) return (d[0] == 0 || (d[0] == '0' && d[1] == 0)) ? std::string() : std::string(d);
  if (const char* x = getenv("XDG_CACHE_HOME"); x && x[0]) return std::string(x) + "/mythgpu/jit";
  if (const char* h = getenv("HOME"); h && h[0]) return std::string(h) + "/.cache/mythgpu/jit";
  return std::string();
}

uint64_t key_hash(const std::string& s, uint64_t seed) {
  uint64_t h = 0xCBF29CE484222325ull ^ seed;
  for (unsigned char c : s) h = (h ^ c) * 0x100000001B3ull;
  h ^= h >> 33;
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  return h;
}

std::string compile_key(const std::string& src) {
  std::string k = src;
  k += "\n//mythgpu-jit-key\n";
  for (char** e = environ; e && *e; e++)
    if ((!std::strncmp(*e, "AMD_COMGR_", 10) || !std::strncmp(*e, "MYTHGPU_JIT", 11)) &&
        std::strncmp(*e, "MYTHGPU_JIT_DISK_CACHE=", 23) && std::strncmp(*e, "MYTHGPU_JIT_CACHE=", 18) &&
        std::strncmp(*e, "MYTHGPU_JIT_TIMING=", 19) && std::strncmp(*e, "MYTHGPU_JITD=", 13) &&
        std::strncmp(*e, "AMD_COMGR_CACHE", 15)) {
      k += *e;
      k.push_back('\n');
    }
  k += "isolate=" + std::to_string(isolated() ? 1 : 0) + "\n";
  k += "hip=" + std::to_string(HIP_VERSION) + " built=" __DATE__ " " __TIME__ "\n";
  return k;
}

bool mkdirs(const std::string& dir) {
  for (size_t p = 1; p <= dir.size(); p++) {
    if (p == dir.size() || dir[p] == '/') {
      const std::string part = dir.substr(0, p);
      if (mkdir(part.c_str(), 0700) != 0 && errno != EEXIST) return false;
    }
  }
  return true;
}

bool disk_load(const std::string& path, uint64_t klen, uint64_t h1, std::vector<char>& code) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  uint64_t hdr[3] = {0, 0, 0};
  bool ok = fread(hdr, 8, 3, f) == 3 && hdr[0] == kCoMagic && hdr[1] == klen && hdr[2] == h1;
  if (ok) {
    fseek(f, 0, SEEK_END);
    const long end = ftell(f);
    ok = end > 24 + 4;
    if (ok) {
      std::vector<char> buf((size_t)end - 24);
      fseek(f, 24, SEEK_SET);
      ok = fread(buf.data(), 1, buf.size(), f) == buf.size() && !std::memcmp(buf.data(), "\x7f" "ELF", 4);
      if (ok) code.swap(buf);
    }
  }
  fclose(f);
  return ok;
}

void disk_store(const std::string& dir, const std::string& path, uint64_t klen, uint64_t h1,
                const std::vector<char>& code) {
  if (!mkdirs(dir)) return;
  static std::atomic<uint64_t> seq{0};
  const std::string tmp = path + ".tmp." + std::to_string(getpid()) + "." + std::to_string(seq++);
  FILE* f = fopen(tmp.c_str(), "wb");
  if (!f) return;
  const uint64_t hdr[3] = {kCoMagic, klen, h1};
  const bool ok = fwrite(hdr, 8, 3, f) == 3 && fwrite(code.data(), 1, code.size(), f) == code.size();
  if (fclose(f) == 0 && ok && rename(tmp.c_str(), path.c_str()) == 0) return;
  (void)unlink(tmp.c_str());
}

std::string disk_path(const std::string& dir, const std::string& key) {
  char name[40];
  snprintf(name, sizeof name, "%016llx%016llx.co", (unsigned long long)key_hash(key, 0),
           (unsigned long long)key_hash(key, 0x9E3779B97F4A7C15ull));
  return dir + "/" + name;
}

}  // namespace

// ---------------------------------------------------------------------------
// Load gate: read the AMDHSA kernel descriptors of a code object (ELF64, EM_AMDGPU).  Each kernel
// `k` has a 64-byte descriptor at symbol `k.kd`: group_segment_fixed_size at +0,
// private_segment_fixed_size at +4, kernel_code_properties (u16) at +56, whose bit 11 is
// USES_DYNAMIC_STACK.  These are the fields the runtime sizes scratch from, so they are what a
// load has to be judged by (the msgpack metadata note only restates them).
// ---------------------------------------------------------------------------
namespace {
std::atomic<uint64_t> g_refused{0};

template <typename T>
bool read_at(const std::vector<uint8_t>& b, size_t off, T& v) {
  if (off > b.size() || b.size() - off < sizeof(T)) return false;
  std::memcpy(&v, b.data() + off, sizeof(T));
  return true;
}
}  // namespace

int code_object_info(const void* code, size_t len, CodeObjectInfo& out, std::string& err) {
  out = CodeObjectInfo{};
  if (!code || len < sizeof(Elf64_Ehdr)) {
    err = "code object too short";
    return MG_E_INVALID;
  }
  const std::vector<uint8_t> b((const uint8_t*)code, (const uint8_t*)code + len);
  Elf64_Ehdr eh;
  std::memcpy(&eh, b.data(), sizeof eh);
  if (std::memcmp(eh.e_ident, ELFMAG, SELFMAG) || eh.e_ident[EI_CLASS] != ELFCLASS64 || eh.e_machine != EM_AMDGPU ||
      eh.e_shentsize != sizeof(Elf64_Shdr)) {
    err = "not an AMDGPU ELF64 code object";
    return MG_E_INVALID;
  }
  std::vector<Elf64_Shdr> sh(eh.e_shnum);
  for (size_t i = 0; i < sh.size(); i++)
    if (!read_at(b, eh.e_shoff + i * sizeof(Elf64_Shdr), sh[i])) {
      err = "section headers out of range";
      return MG_E_INVALID;
    }
  // prefer .symtab (every symbol); a stripped object still has .dynsym with the .kd symbols
  int symi = -1;
  for (size_t i = 0; i < sh.size(); i++)
    if (sh[i].sh_type == SHT_SYMTAB) symi = (int)i;
  if (symi < 0)
    for (size_t i = 0; i < sh.size(); i++)
      if (sh[i].sh_type == SHT_DYNSYM) symi = (int)i;
  if (symi < 0 || sh[symi].sh_link >= sh.size() || sh[symi].sh_entsize != sizeof(Elf64_Sym)) {
    err = "no symbol table";
    return MG_E_INVALID;
  }
  const Elf64_Shdr& st = sh[symi];
  const Elf64_Shdr& strs = sh[st.sh_link];
  for (uint64_t k = 0; k < st.sh_size / sizeof(Elf64_Sym); k++) {
    Elf64_Sym s;
    if (!read_at(b, st.sh_offset + k * sizeof(Elf64_Sym), s)) break;
    if (s.st_name >= strs.sh_size || s.st_shndx == SHN_UNDEF || s.st_shndx >= sh.size()) continue;
    const size_t noff = strs.sh_offset + s.st_name;
    if (noff >= b.size()) continue;
    const char* nm = (const char*)b.data() + noff;
    const size_t nl = strnlen(nm, b.size() - noff);
    const Elf64_Shdr& sec = sh[s.st_shndx];
    if (nl == 17 && !std::strncmp(nm, "mgj_meta_eval_cpb", 17)) {  // jit_asm.cpp: the solo eval kernel's grid
      if (s.st_value < sec.sh_addr || s.st_value + 4 > sec.sh_addr + sec.sh_size ||
          !read_at(b, sec.sh_offset + (s.st_value - sec.sh_addr), out.eval_cpb)) {
        err = "mgj_meta_eval_cpb outside its section";
        return MG_E_INVALID;
      }
      continue;
    }
    if (nl < 4 || std::strncmp(nm + nl - 3, ".kd", 3)) continue;
    if (s.st_value < sec.sh_addr || s.st_value + 64 > sec.sh_addr + sec.sh_size) {
      err = "kernel descriptor outside its section";
      return MG_E_INVALID;
    }
    const size_t off = sec.sh_offset + (s.st_value - sec.sh_addr);
    uint32_t group = 0, priv = 0;
    uint16_t props = 0;
    if (!read_at(b, off, group) || !read_at(b, off + 4, priv) || !read_at(b, off + 56, props)) {
      err = "kernel descriptor out of range";
      return MG_E_INVALID;
    }
    out.kernels++;
    out.max_private_bytes = std::max(out.max_private_bytes, priv);
    out.max_group_bytes = std::max(out.max_group_bytes, group);
    if (props & (1u << 11)) out.dynamic_stack = true;
  }
  if (!out.kernels) {
    err = "no kernel descriptors";
    return MG_E_INVALID;
  }
  return MG_OK;
}

int code_object_gate(const CodeObjectInfo& ci, std::string& why) {
  static const uint32_t cap = [] {
    const char* c = getenv("MYTHGPU_JIT_PRIVATE_CAP");
    return c ? (uint32_t)strtoul(c, nullptr, 0) : 16384u;
  }();
  if (ci.dynamic_stack) {
    why = "code object refused: a kernel uses a dynamic stack";
    return MG_E_UNSUPPORTED;
  }
  if (ci.max_private_bytes > cap) {
    why = "code object refused: " + std::to_string(ci.max_private_bytes) + " B of private segment per lane (cap " +
          std::to_string(cap) + ", MYTHGPU_JIT_PRIVATE_CAP)";
    return MG_E_UNSUPPORTED;
  }
  if (ci.max_group_bytes > 160u * 1024u) {
    why = "code object refused: " + std::to_string(ci.max_group_bytes) + " B of LDS (gfx950 has 160 KiB per CU)";
    return MG_E_UNSUPPORTED;
  }
  return MG_OK;
}

int jit_check_code_object(const std::vector<char>& code, std::string& why) {
  CodeObjectInfo ci;
  std::string err;
  int rc = code_object_info(code.data(), code.size(), ci, err);
  if (rc == MG_OK) {
    rc = code_object_gate(ci, why);
  } else {
    why = "code object refused: " + err;
    rc = MG_E_UNSUPPORTED;
  }
  if (rc != MG_OK) g_refused++;
  return rc;
}

uint64_t jit_refused_total() { return g_refused.load(); }

void jit_disk_evict(const std::string& src) {
  const std::string dir = disk_cache_dir();
  if (dir.empty()) return;
  (void)unlink(disk_path(dir, compile_key(src)).c_str());
}

int jit_compile(const std::string& src, std::vector<char>& code, std::string& log, bool* from_disk) {
  const std::string dir = disk_cache_dir();
  const bool timing = getenv("MYTHGPU_JIT_TIMING") != nullptr;
  std::string path;
  uint64_t klen = 0, h1 = 0;
  if (from_disk) *from_disk = false;
  if (!dir.empty()) {
    const std::string key = compile_key(src);
    klen = key.size();
    h1 = key_hash(key, 0);
    path = disk_path(dir, key);
    if (disk_load(path, klen, h1, code)) {
      if (timing) fprintf(stderr, "mythgpu: JIT code object from the disk cache %s\n", path.c_str());
      if (int rc = jit_check_code_object(code, log)) {  // written by a build without the gate
        (void)unlink(path.c_str());
        code.clear();
        return rc;
      }
      if (from_disk) *from_disk = true;
      return MG_OK;
    }
  }
  int rc = MG_E_UNSUPPORTED;
  bool done = false;
  if (isolated()) {
    bool available = true;
    rc = helper_compile(src, code, log, available);
    done = available;
    if (!available) {
      static std::once_flag warn;
      std::call_once(warn, [&] { fprintf(stderr, "mythgpu: %s; compiling in-process\n", helper().why.c_str()); });
    }
  }
  if (!done) rc = jit_compile_local(src, code, log);
  if (rc == MG_OK) {
    rc = jit_check_code_object(code, log);
    if (rc != MG_OK) {
      if (timing) fprintf(stderr, "mythgpu: %s\n", log.c_str());
      code.clear();
      return rc;
    }
  }
  if (rc == MG_OK && !path.empty()) {
    disk_store(dir, path, klen, h1, code);
    if (timing) fprintf(stderr, "mythgpu: JIT code object stored in the disk cache %s\n", path.c_str());
  }
  return rc;
}

int jit_compile_local(const std::string& src, std::vector<char>& code, std::string& log) {
  const char* which = getenv("MYTHGPU_JIT_COMPILER");
  const bool use_rtc = which && std::strcmp(which, "hiprtc") == 0;
  int rc;
  const bool is_asm = src.compare(0, std::strlen(kAsmMarker), kAsmMarker) == 0;
  if (is_asm) {
    if (!comgr().ok) {
      log = "comgr not available (the assembly tier needs it)";
      return MG_E_UNSUPPORTED;
    }
    rc = comgr_assemble(src, code, log);
  } else if (!use_rtc && comgr().ok) {
    rc = comgr_compile(src, code, log);
  } else {
    rc = hiprtc_compile(src, code, log);
  }
  if (rc != MG_OK) return rc;
  // MYTHGPU_JIT_DUMP=<prefix>: keep the source and code object for offline disassembly
  if (const char* dump = getenv("MYTHGPU_JIT_DUMP")) {
    const std::string base(dump);
    if (FILE* f = fopen((base + (is_asm ? ".s" : ".hip")).c_str(), "wb")) {
      fwrite(src.data(), 1, src.size(), f);
      fclose(f);
    }
    if (FILE* f = fopen((base + ".co").c_str(), "wb")) {
      fwrite(code.data(), 1, code.size(), f);
      fclose(f);
    }
  }
  return MG_OK;
}

}  // namespace mg
