// JIT first tier: gfx950 assembly emitted straight from the specialised program.
//
// The HIP-source JIT (jit.cpp) costs ~140 ms of clang + LLVM per query on the box's host
// (profiles/r04a_jit_phases.jsonl: C2 front end + optimiser 54 ms, machine code generation
// 84 ms), longer than a hard query's whole search.  This emitter writes the same search kernel
// (mgj_search; mgj_gen for per-candidate verdicts) as GCN assembly with its own register
// allocation, so a compile is the emission (well under a millisecond) plus an assembler pass and
// a link (comgr, a few ms).  The O3 kernel still compiles behind it and replaces it on the same
// index stream (search.search); both compute the verdict of every index exactly as the
// interpreter and the C port do (GEN3, include/mythgpu.h).
//
// Model of the code:
//  * one wave = one aligned group of 64 candidate indices; EXEC stays all-ones inside the body
//    (every choice the generator makes per group is an SGPR branch, every per-lane choice a
//    v_cndmask), so no structurisation is needed;
//  * a value of width w is ceil(w/32) limbs, each a literal or a VGPR (copies are aliases:
//    VGPRs are reference-counted); limbs no user reads are never computed (demanded limbs,
//    backward pass); a Bool is a 64-lane mask in an SGPR pair (compares write masks, ASSERT
//    ANDs them into the verdict mask, ITE selects through VCC);
//  * VCC carries the add/sub chains; gfx950 needs two wait states between a VALU write of an
//    SGPR (VCC, a compare's mask) and a VALU read of it, which the emitter counts and pads with
//    s_nop (LLVM's GCNHazardRecognizer does the same); a branch target is treated as a fresh
//    write of every such SGPR;
//  * no scalar stores and no scalar-cache writes anywhere: results leave through vector atomics.
//
// The tier covers LASER's whole vocabulary (round 5: symbolic UDIV/UREM/SDIV/SREM/SMOD, variable
// shifts, EXP, Keccak-256, UMUL_NOOVF).  What it still refuses (MG_E_UNSUPPORTED: the search stays
// on the interpreter until the O3 kernel is ready, an eval goes to the O3 kernel) is a kernel whose
// live values do not fit 256 VGPRs plus the LDS spill slots of one wave (Gen::spill_one, `solo`),
// and values wider than the limb bound (kMaxLimbs).
#include <algorithm>
#include <array>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "jit.hpp"

namespace mg {

namespace {

struct AsmFail {
  std::string why;
};
[[noreturn]] void fail(const std::string& w) { throw AsmFail{w}; }

inline uint32_t Lw(uint32_t w) { return (w + 31) / 32; }
inline uint32_t topmask(uint32_t w) { return (w & 31) ? ((1u << (w & 31)) - 1u) : 0xFFFFFFFFu; }
inline uint32_t gsalt(uint32_t c, uint32_t j) { return c * 0x9E3779B9u + j * 0x85EBCA6Bu + 0x27D4EB2Fu; }

constexpr int kVCC = 106;  // vcc_lo in the hazard table (vcc_hi = 107)
constexpr uint32_t kMaxLimbs = 64;

enum LKind : uint8_t { LU, LL, LR };
struct Limb {
  LKind k = LU;
  uint32_t v = 0;
  uint32_t g = 0;  // allocation tag of an allocated VGPR (Emitter::vgen), checked under MYTHGPU_JIT_ASM_CHECK
  bool lit() const { return k == LL; }
  bool reg() const { return k == LR; }
  bool operator==(const Limb& o) const { return k == o.k && v == o.v; }
};
inline Limb Lit(uint32_t x) { return Limb{LL, x}; }
inline Limb Reg(uint32_t r) { return Limb{LR, r}; }

// a 64-lane Bool: literal (all lanes equal) or an SGPR pair
struct Mask {
  int k = 0;  // 0 none, 1 literal, 2 pair
  bool ones = false;
  int s = -1;
};

struct Val {
  std::vector<Limb> l;
  Mask m;
  uint32_t w = 0;
  bool def = false;
};

std::string hexs(uint32_t x) {
  char b[16];
  snprintf(b, sizeof b, "0x%x", x);
  return b;
}
// an integer operand: inline constants (-16..64) as decimal, others as a 32-bit literal
bool inl(uint32_t x) {
  const int32_t s = (int32_t)x;
  return s >= -16 && s <= 64;
}
std::string imm(uint32_t x) { return inl(x) ? std::to_string((int32_t)x) : hexs(x); }
std::string V(uint32_t r) { return "v" + std::to_string(r); }
std::string S(uint32_t r) { return "s" + std::to_string(r); }
std::string SP(uint32_t r) { return "s[" + std::to_string(r) + ":" + std::to_string(r + 1) + "]"; }
std::string VP(uint32_t r) { return "v[" + std::to_string(r) + ":" + std::to_string(r + 1) + "]"; }

// fixed registers
// VGPRs: v0 tid, v1 lane, v2/v3 lane key (lo/hi), v4/v5 group-lane key K (lo/hi), v6 zero, v7 scratch,
//        v[8:9] 64-bit scratch, v10/v11 the group keys of the wave's next 64 groups (search kernels:
//        lane l holds G of the l-th, lo/hi); the allocator hands out v12 and up
// SGPRs: s[0:1] kernarg, s2 block id, s3 wave in block, s[4:5] gconsts, s[8:9] start, s[10:11] count,
//        s[12:13] sk, s[14:15] sg, s[16:17] hit / verdict_out, s18 flags, s19 nblk, s[20:21] a0,
//        s[22:23] end, s[24:25] ngroups, s[26:27] g, s28 gstride, s29 early, s[30:31] wave best,
//        s[32:33] wave hits, s[34:35] gbase, s[36:37] G, s[38:39] verdict, s[40:41] temps,
//        s[42:43] ~0 unless the launch stops early, s[10:11] / s[12:13] the call's partial first / last
//        group base (after the prologue), s7 the next group's lane in v10/v11; pairs s[44:45] ..
//        s[98:99] allocated
constexpr int kV0 = 12;
constexpr int kS0 = 44, kS1 = 100;

class Emitter {
 public:
  std::ostringstream o;
  int64_t pos = 0;
  std::map<int, int64_t> vw;  // SGPR -> position of its last VALU write
  int nlab = 0;
  std::vector<int> vref = std::vector<int>(256, 0);
  // MYTHGPU_JIT_ASM_CHECK=1: every allocation of a VGPR gets a fresh tag, every limb the tag of the
  // allocation it was computed into; a read, retain or release of a limb whose register has since
  // been released or handed out again fails the emission (a lifetime bug of the allocator, which
  // would otherwise read another value's register in the kernel)
  std::vector<uint32_t> vgen = std::vector<uint32_t>(256, 0);
  uint32_t gen_ctr = 0;
  static bool check_on() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_CHECK");
      return g && g[0] == '1';
    }();
    return on;
  }
  void check(const Limb& l) const {
    if (!check_on() || !l.reg() || (int)l.v < vfirst) return;
    if (l.g == 0) fail("internal: an allocated VGPR v" + std::to_string(l.v) + " without its allocation tag");
    if (vref[l.v] <= 0 || vgen[l.v] != l.g)
      fail("internal: v" + std::to_string(l.v) + " used after its register was released or reallocated");
  }
  int vfirst = kV0;  // the allocator's first VGPR: below it the fixed registers and the literal pool
  int vhigh = kV0;
  std::vector<int> sref = std::vector<int>(kS1, 0);
  int shigh = kS0;

  // --- instruction streams with the gfx950 VALU-SGPR hazard --------------------------------
  void valu(const std::string& s, std::initializer_list<int> rd = {}, std::initializer_list<int> wr = {}) {
    int64_t need = 0;
    for (int r : rd) {
      auto it = vw.find(r);
      if (it != vw.end()) need = std::max(need, it->second + 3 - pos);
    }
    if (need > 0) {
      o << "  s_nop " << (need - 1) << "\n";
      pos += need;
    }
    o << "  " << s << "\n";
    pos++;
    for (int r : wr) vw[r] = pos - 1;
  }
  // SGPR pair s..s+1 written by a VALU within the last two instructions (a VALU read would wait)
  bool fresh_valu_write(int s) const {
    for (int r : {s, s + 1}) {
      auto it = vw.find(r);
      if (it != vw.end() && it->second + 3 - pos > 0) return true;
    }
    return false;
  }
  void salu(const std::string& s, std::initializer_list<int> wr = {}) {
    o << "  " << s << "\n";
    pos++;
    for (int r : wr) vw.erase(r);
  }
  // memory / wait / branch instructions: no wait-state credit; a VMEM reading an SGPR a VALU wrote
  // needs five
  void mem(const std::string& s, std::initializer_list<int> rd = {}) {
    int64_t need = 0;
    for (int r : rd) {
      auto it = vw.find(r);
      if (it != vw.end()) need = std::max(need, it->second + 6 - pos);
    }
    if (need > 0) {
      o << "  s_nop " << (need - 1) << "\n";
      pos += need;
    }
    o << "  " << s << "\n";
  }
  void ctl(const std::string& s) {
    // a pending dictionary read does not cross a branch or a label: the waits are placed along one path
    if (!lds_pending.empty()) {
      if (s.compare(0, 9, "s_branch ") == 0 || s.compare(0, 10, "s_cbranch_") == 0) lds_flush();
      else if (s.compare(0, 9, "s_waitcnt") == 0 && s.find("lgkmcnt(0)") != std::string::npos) lds_pending.clear();
    }
    o << "  " << s << "\n";
  }
  std::string newlab() { return ".Lm" + std::to_string(nlab++); }
  int label_events = 0;  // labels emitted so far: SGPR state tracked at emission time is void past one
  void label(const std::string& L) {
    lds_flush();
    label_events++;
    o << L << ":\n";
    for (auto& kv : vw) kv.second = std::max(kv.second, pos - 1);
  }
  static std::initializer_list<int> none() { return {}; }

  // --- VGPRs ---------------------------------------------------------------------------------
  // VGPRs a dictionary's LDS reads are still filling: the wave waits (s_waitcnt lgkmcnt(0)) only when
  // one of them is next named — read, written or reallocated — not right after the reads, so the LDS
  // latency overlaps the generator's other work (Gen::VL, valloc, lds_flush at the body's end)
  std::set<int> lds_pending;
  void lds_flush() {
    if (lds_pending.empty()) return;
    ctl("s_waitcnt lgkmcnt(0)");
    lds_pending.clear();
  }
  std::function<bool()> on_pressure;  // drop cached values (value numbering); true if any went
  std::function<bool()> on_hard;      // all 256 taken and no cache entry left: spill a value (eval)
  // The value caches may not raise the kernel's VGPR count past the occupancy step the kernel
  // reaches without them (jit_asm_source): an allocation at or above vsoft first drops the caches.
  // (C4: the literal cache alone took the search kernel from 98 to 134 VGPRs, 4 to 3 waves per SIMD.)
  int vsoft = 256;
  int vhard = 256;  // the register file's end (MYTHGPU_JIT_ASM_SPILL_TEST lowers it to exercise spills)
  uint32_t valloc() {
    for (;;) {
      int r = vfirst;
      while (r < vhard && vref[r]) r++;
      // cache entries go one at a time (least recently used first) until a register below the limit
      // is free or the caches are empty
      if ((r >= 256 || r >= vsoft) && on_pressure && on_pressure()) continue;
      if (r >= vhard && on_hard && on_hard()) continue;
      if (r >= vhard) fail("out of VGPRs");
      if (lds_pending.count(r)) lds_flush();  // a register whose load is still in flight
      vref[r] = 1;
      vgen[r] = ++gen_ctr;
      vhigh = std::max(vhigh, r + 1);
      return (uint32_t)r;
    }
  }
  // an even-aligned register pair (64-bit VGPR operands), each half with its own reference
  uint32_t valloc2() {
    for (;;) {
      int r = (vfirst + 1) & ~1;
      while (r + 1 < vhard && (vref[r] || vref[r + 1])) r += 2;
      if ((r + 1 >= 256 || r + 1 >= vsoft) && on_pressure && on_pressure()) continue;
      if (r + 1 >= vhard && on_hard && on_hard()) continue;
      if (r + 1 >= vhard) fail("out of VGPRs");
      if (lds_pending.count(r) || lds_pending.count(r + 1)) lds_flush();
      for (int q = 0; q < 2; q++) {
        vref[r + q] = 1;
        vgen[r + q] = ++gen_ctr;
      }
      vhigh = std::max(vhigh, r + 2);
      return (uint32_t)r;
    }
  }
  void retain(const Limb& l) {
    check(l);
    if (l.reg() && (int)l.v >= vfirst) vref[l.v]++;
  }
  std::function<void(uint32_t)> on_free;  // a register's allocation tag died (limb value numbering)
  void release(const Limb& l) {
    check(l);
    if (l.reg() && (int)l.v >= vfirst) {
      if (--vref[l.v] < 0) fail("internal: VGPR released twice");
      if (vref[l.v] == 0 && on_free) on_free(vgen[l.v]);
    }
  }
  // --- SGPR pairs ----------------------------------------------------------------------------
  int sfree() const {  // SGPR pairs free
    int n = 0;
    for (int r = kS0; r + 1 < kS1; r += 2) n += !sref[r];
    return n;
  }
  std::function<bool()> on_spressure;  // move a Bool value's mask to its VGPR form; true if one went
  int salloc() {
    for (;;) {
      for (int r = kS0; r + 1 < kS1; r += 2)
        if (!sref[r]) {
          sref[r] = 1;
          shigh = std::max(shigh, r + 2);
          return r;
        }
      if (!on_spressure || !on_spressure()) break;
    }
    fail("out of SGPRs");
  }
  void sretain(const Mask& m) {
    if (m.k == 2) sref[m.s]++;
  }
  void srelease(const Mask& m) {
    if (m.k == 2 && --sref[m.s] < 0) fail("internal: SGPR pair released twice");
  }
};

struct Gen {
  const Lowered& P;
  const std::vector<GenSpec>& specs;
  const std::vector<uint32_t>& G;  // generator constants
  mutable Emitter E;  // (mutable: naming a register may first wait for its pending LDS read)
  std::vector<Val> val;
  std::vector<uint64_t> need;        // demanded limbs per value id (bit j = limb j)
  std::vector<int32_t> last;         // last vcode index reading each value id
  std::map<uint32_t, uint32_t> cval; // coordinate -> value id of its (latest) generated value
  std::vector<int32_t> def;          // value id -> defining vcode index
  std::vector<uint32_t> copysrc;     // vcode index of a MIXED K_COORD -> its COPY source's value id
  bool gen_kernel = false;           // mgj_gen (verdict bytes) instead of mgj_search
  bool eval_kernel = false;          // mgj_eval: coordinates from HBM-resident SoA rows (no generator)
  // Dictionary tables staged in LDS by the prologue, limb-major ([limb][entry], so lanes that drew
  // different entries hit different banks): a gather is then one ds_read per limb instead of a
  // global load whose latency the wave waits out (18 VMEM reads per group on C2 before this)
  std::map<uint32_t, uint32_t> lds_base;  // gconsts offset of a table -> LDS word offset
  std::map<uint32_t, std::pair<uint32_t, uint32_t>> lds_shape;  // table -> (entries, limbs)
  uint32_t lds_words = 0;
  static constexpr uint32_t kLdsWords = 8192;  // 32 KiB per 256-lane block

  std::vector<Instr> code;            // the program in emission order (reorder())
  Gen(const Lowered& p, const std::vector<GenSpec>& s, const std::vector<uint32_t>& g)
      : P(p), specs(s), G(g), val(p.vwidth.size()), need(p.vwidth.size(), 0), last(p.vwidth.size(), -1),
        def(p.vwidth.size(), -1), code(p.vcode) {}

  // Emission order: every ASSERT / WATCH in program order, each preceded by the instructions it
  // needs that are not emitted yet (operands first, depth-first).  A value is then computed just
  // before its first use and a later constraint's work comes after an earlier one's early exit:
  // shorter live ranges (C4's eval program peaked at 220 live VGPRs in program order) and less
  // work per rejected group.  Verdicts do not depend on the order (an AND of the asserts).
  void reorder() {
    const std::vector<Instr>& v = P.vcode;
    std::vector<int32_t> dix(P.vwidth.size(), -1);
    for (size_t k = 0; k < v.size(); k++)
      if (v[k].dst != MG_NONE && v[k].dst < dix.size() && dix[v[k].dst] < 0) dix[v[k].dst] = (int32_t)k;
    std::map<uint32_t, int32_t> coord_at;  // coordinate -> its first K_COORD
    for (size_t k = 0; k < v.size(); k++)
      if (v[k].op == K_COORD && !coord_at.count(v[k].p0)) coord_at[v[k].p0] = (int32_t)k;
    auto operands = [&](const Instr& in, std::vector<int32_t>& out) {
      out.clear();
      auto add = [&](uint32_t id) {
        if (id != MG_NONE && id < dix.size() && dix[id] >= 0) out.push_back(dix[id]);
      };
      switch (in.op) {
        case K_CONST: break;
        case K_COORD:
          if (!eval_kernel && in.p0 < specs.size()) {
            const GenSpec& sp = specs[in.p0];
            if ((sp.kind & 0xFFu) == MG_GEN_MIXED && sp.p[3] != MG_NONE && (sp.p[2] & 0xFFFFu)) {
              auto it = coord_at.find(sp.p[3]);
              if (it != coord_at.end()) out.push_back(it->second);
            }
          }
          break;
        case K_LOOKUP:
          add(in.a);
          add(in.p0);
          for (uint32_t q = 0; q < 2 * in.c; q++) add(P.vaux[in.p1 + q]);
          break;
        case K_NOT: case K_NEG: case K_EXTRACT: case K_ZEXT: case K_SEXT: case K_ASSERT: case K_COPY: case K_WATCH:
          add(in.a);
          break;
        case K_ITE:
          add(in.a);
          add(in.b);
          add(in.c);
          break;
        default:
          add(in.a);
          add(in.b);
          break;
      }
    };
    std::vector<char> done(v.size(), 0);
    std::vector<Instr> out;
    out.reserve(v.size());
    std::vector<int32_t> ops;
    auto visit = [&](int32_t root) {
      std::vector<std::pair<int32_t, size_t>> st{{root, 0}};  // (instruction, next operand)
      std::vector<std::vector<int32_t>> opl;
      opl.emplace_back();
      operands(v[root], opl.back());
      while (!st.empty()) {
        auto& top = st.back();
        if (done[top.first]) {
          st.pop_back();
          opl.pop_back();
          continue;
        }
        if (top.second < opl.back().size()) {
          const int32_t o = opl.back()[top.second++];
          if (!done[o]) {
            st.push_back({o, 0});
            opl.emplace_back();
            operands(v[o], opl.back());
          }
          continue;
        }
        done[top.first] = 1;
        out.push_back(v[top.first]);
        st.pop_back();
        opl.pop_back();
      }
    };
    if (eval_kernel && greedy_on()) {
      greedy_roots(v, operands, done, visit);
    } else if (!eval_kernel && heavy_last_on()) {
      heavy_last_roots(v, operands, done, visit);
    } else {
      for (size_t k = 0; k < v.size(); k++)
        if (v[k].op == K_ASSERT || v[k].op == K_WATCH) visit((int32_t)k);
    }
    for (size_t k = 0; k < v.size(); k++)
      if (!done[k]) visit((int32_t)k);
    code.swap(out);
  }
  // Search kernels: constraints whose not-yet-emitted cone holds a heavy operator (Keccak, EXP,
  // division: hundreds to thousands of VALU per candidate) go after the light ones.  The early exit after each ASSERT
  // (an early-exit search's wave leaves once all 64 of its candidates failed) then skips the heavy
  // work of most rejected groups: a query whose cheap constraint rejects most candidates ahead of a
  // Keccak (bench's C5 hard query: the ~2^-8 needle behind two Keccak-f[1600]) no longer pays the
  // Keccaks for them.  Light constraints keep program order; the heavy ones follow, cheapest
  // remaining cone first.  Verdicts do not depend on the order; a full-evaluation launch (no early
  // exit) does the same work in another order.  MYTHGPU_JIT_ASM_HEAVY_LAST=0: program order.
  static bool heavy_last_on() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_HEAVY_LAST");
      return !(g && g[0] == '0');
    }();
    return on;
  }
  // rough VALU per candidate of one instruction (to order the heavy cones, cheapest first)
  uint32_t op_weight(const Instr& in) const {
    const uint32_t w = (in.dst != MG_NONE && in.dst < P.vwidth.size()) ? P.vwidth[in.dst] : 32u;
    const uint32_t L = std::max(1u, Lw(std::max(w, in.op >= K_EQ && in.op <= K_UMUL_NOOVF ? in.p1 : w)));
    switch (in.op) {
      case K_KECCAK: return 2500u * (in.p0 / 136u + 1u);
      case K_EXP: return 1500u;
      case K_UDIV: case K_UREM: case K_SDIV: case K_SREM: case K_SMOD: return 600u;
      case K_MUL: return 4u * L * L;
      case K_UMUL_NOOVF: return 8u * L * L;
      case K_SHL: case K_LSHR: case K_ASHR: return 4u * L;
      case K_LOOKUP: return 2u * Lw(in.b) * std::max(1u, in.c);
      case K_COORD: return 8u * L;
      default: return L;
    }
  }
  static bool heavy_op(uint32_t op) {
    return op == K_KECCAK || op == K_EXP || op == K_UDIV || op == K_UREM || op == K_SDIV || op == K_SREM || op == K_SMOD;
  }
  template <class Ops, class Visit>
  void heavy_last_roots(const std::vector<Instr>& v, Ops& operands, const std::vector<char>& done, Visit& visit) {
    std::vector<int32_t> roots;
    for (size_t k = 0; k < v.size(); k++)
      if (v[k].op == K_ASSERT) roots.push_back((int32_t)k);
    std::vector<int32_t> mark(v.size(), -1), st, ops;
    int32_t stamp = 0;
    auto cone_cost = [&](int32_t r, bool& heavy) -> uint64_t {  // the not-yet-emitted cone of r
      uint64_t c = 0;
      heavy = false;
      st.assign(1, r);
      mark[r] = ++stamp;
      while (!st.empty()) {
        const int32_t x = st.back();
        st.pop_back();
        c += op_weight(v[x]);
        heavy = heavy || heavy_op(v[x].op);
        operands(v[x], ops);
        for (int32_t o : ops)
          if (!done[o] && mark[o] != stamp) {
            mark[o] = stamp;
            st.push_back(o);
          }
      }
      return c;
    };
    std::vector<char> taken(roots.size(), 0);
    for (size_t step = 0; step < roots.size(); step++) {
      size_t pick = roots.size();
      uint64_t best = UINT64_MAX;
      for (size_t i = 0; i < roots.size(); i++) {
        if (taken[i]) continue;
        bool heavy = false;
        const uint64_t c = cone_cost(roots[i], heavy);
        if (!heavy) {  // the first light constraint in program order
          pick = i;
          break;
        }
        if (c < best) {
          best = c;
          pick = i;
        }
      }
      taken[pick] = 1;
      visit(roots[pick]);
    }
  }
  // MYTHGPU_JIT_ASM_GREEDY=1: the eval kernel's constraints in greedy order (below).  Opt-in: it lowers
  // C4's cache-free peak (238 -> 208 VGPRs) but the kernel's time did not move (the caches fill the
  // occupancy step either way; profiles/r05i_eval_glds.jsonl), and with the model watch rows as roots
  // it ran C4's read-back kernel out of registers
  static bool greedy_on() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_GREEDY");
      return g && g[0] == '1';
    }();
    return on;
  }
  // The eval kernel evaluates every constraint (no early exit), so their order is free: each step
  // emits the constraint whose not-yet-emitted cone leaves the fewest limbs live — the limbs of
  // cone values still read outside it, less the limbs of live values whose last readers are in it
  // (C4: coordinate rows and storage keys loaded early were held across hundreds of constraints
  // that did not read them; 246 live VGPRs in program order)
  template <class Ops, class Visit>
  void greedy_roots(const std::vector<Instr>& v, Ops& operands, const std::vector<char>& done, Visit& visit) {
    const size_t n = v.size();
    std::vector<std::vector<int32_t>> opl(n);
    std::vector<int32_t> users(n, 0);  // readers not yet emitted
    for (size_t k = 0; k < n; k++) {
      operands(v[k], opl[k]);
      std::sort(opl[k].begin(), opl[k].end());
      opl[k].erase(std::unique(opl[k].begin(), opl[k].end()), opl[k].end());
      for (int32_t o : opl[k]) users[o]++;
    }
    auto limbs_of = [&](int32_t k) -> int32_t {
      const Instr& in = v[k];
      if (in.op == K_CONST || in.dst == MG_NONE || in.dst >= P.vwidth.size()) return 0;
      const uint32_t w = P.vwidth[in.dst];
      return w <= 1 ? 0 : (int32_t)Lw(w);
    };
    std::vector<int32_t> roots;
    for (size_t k = 0; k < n; k++)
      if (v[k].op == K_ASSERT || v[k].op == K_WATCH) roots.push_back((int32_t)k);
    std::vector<int32_t> mark(n, -1), inner(n, 0);  // cone membership stamp; readers inside the cone
    std::vector<int32_t> cone, st;
    int32_t stamp = 0;
    auto gather = [&](int32_t r) {  // the not-yet-emitted cone of r into `cone`, reader counts into inner
      cone.clear();
      st.assign(1, r);
      mark[r] = ++stamp;
      while (!st.empty()) {
        const int32_t x = st.back();
        st.pop_back();
        cone.push_back(x);
        for (int32_t o : opl[x]) {
          if (done[o]) continue;
          if (mark[o] != stamp) {
            mark[o] = stamp;
            st.push_back(o);
          }
        }
      }
      for (int32_t x : cone)
        for (int32_t o : opl[x]) inner[o] = 0;
      for (int32_t x : cone)
        for (int32_t o : opl[x]) inner[o]++;
    };
    std::vector<char> taken(roots.size(), 0);
    for (size_t step = 0; step < roots.size(); step++) {
      int64_t best = INT64_MIN;
      size_t bi = 0;
      for (size_t i = 0; i < roots.size(); i++) {
        if (taken[i]) continue;
        gather(roots[i]);
        int64_t score = 0;
        for (int32_t x : cone) {
          if (users[x] > inner[x]) score -= limbs_of(x);  // read again later: stays live
          for (int32_t o : opl[x])
            if (done[o] && mark[o] != stamp && users[o] == inner[o]) {
              score += limbs_of(o);  // its last readers: freed
              inner[o] = 1 << 30;   // counted once
            }
        }
        if (score > best) {
          best = score;
          bi = i;
        }
      }
      taken[bi] = 1;
      gather(roots[bi]);
      for (int32_t x : cone)
        for (int32_t o : opl[x]) users[o]--;
      visit(roots[bi]);
    }
  }

  // ---------------------------------------------------------------------------------------
  // analysis
  // ---------------------------------------------------------------------------------------
  static uint64_t lowmask(uint32_t n) { return n >= 64 ? ~0ull : ((1ull << n) - 1ull); }
  uint32_t L(uint32_t id) const { return Lw(P.vwidth[id]); }

  const Instr* def_of(uint32_t id) const {
    return (id < def.size() && def[id] >= 0) ? &code[def[id]] : nullptr;
  }

  // bits [p, p + n) of a value of width w -> its limbs
  static uint64_t bit_limbs(uint32_t p, uint32_t n, uint32_t w) {
    if (p >= w || n == 0) return 0;
    const uint32_t e = std::min(w, p + n);
    uint64_t m = 0;
    for (uint32_t q = p / 32; q * 32 < e; q++) m |= 1ull << q;
    return m;
  }

  void analyse() {
    for (uint32_t id = 0; id < P.vwidth.size(); id++)
      if (Lw(P.vwidth[id]) > kMaxLimbs) fail("value wider than 2048 bits");
    if (!getenv("MYTHGPU_JIT_ASM_NOREORDER")) reorder();
    for (size_t k = 0; k < code.size(); k++) {
      const Instr& in = code[k];
      if (in.dst != MG_NONE && in.dst < def.size() && def[in.dst] < 0) def[in.dst] = (int32_t)k;
      switch (in.op) {
        case K_CONST: case K_COORD: case K_ADD: case K_SUB: case K_NEG: case K_AND: case K_OR: case K_XOR:
        case K_NOT: case K_ITE: case K_EQ: case K_ULT: case K_ULE: case K_SLT: case K_SLE: case K_CONCAT:
        case K_EXTRACT: case K_ZEXT: case K_SEXT: case K_LOOKUP: case K_ASSERT: case K_COPY: case K_MUL:
        case K_WATCH: case K_UMUL_NOOVF:
          break;
        case K_UDIV: case K_UREM: case K_SDIV: case K_SREM: case K_SMOD: case K_SHL: case K_LSHR: case K_ASHR:
        case K_EXP:
          // data-dependent operators (widths <= 256 after lowering): div_lit / udivrem / shift_var / exp_var
          if (in.wd > 256) fail("arithmetic wider than 256 bits");
          break;
        case K_KECCAK:
          break;
        default:
          fail("op " + std::to_string(in.op) + " outside the assembly tier");
      }
    }
    // MYTHGPU_JIT_ASM_NO_LDS=1: dictionaries gathered from global memory (diagnostic)
    static const bool no_lds = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_LDS");
      return g && g[0] == '1';
    }();
    if (!eval_kernel && !no_lds) plan_lds();
    // uses (for liveness) and demanded limbs (backward)
    auto use = [&](uint32_t id, size_t k) {
      if (id != MG_NONE && id < last.size()) last[id] = std::max(last[id], (int32_t)k);
    };
    std::map<uint32_t, uint32_t> latest;  // coordinate -> value id, in program order
    copysrc.assign(code.size(), MG_NONE);
    for (size_t k = 0; k < code.size(); k++) {
      const Instr& in = code[k];
      switch (in.op) {
        case K_CONST:
          break;
        case K_WATCH:
          if (eval_kernel) use(in.a, k);  // the eval kernel stores watched values (model read-back)
          break;
        case K_COORD: {
          if (eval_kernel) break;
          // a MIXED coordinate reads its COPY source's value if the program generated it before
          const GenSpec& sp = specs.at(in.p0);
          if ((sp.kind & 0xFFu) == MG_GEN_MIXED && sp.p[3] != MG_NONE && (sp.p[2] & 0xFFFFu)) {
            auto it = latest.find(sp.p[3]);
            if (it != latest.end()) {
              use(it->second, k);
              copysrc[k] = it->second;
            }
          }
          latest[in.p0] = in.dst;
          break;
        }
        case K_LOOKUP:
          use(in.a, k);
          use(in.p0, k);
          for (uint32_t q = 0; q < 2 * in.c; q++) use(P.vaux[in.p1 + q], k);
          break;
        default:
          use(in.a, k);
          if (in.op != K_NOT && in.op != K_NEG && in.op != K_EXTRACT && in.op != K_ZEXT && in.op != K_SEXT &&
              in.op != K_ASSERT && in.op != K_COPY)
            use(in.b, k);
          if (in.op == K_ITE) use(in.c, k);
          break;
      }
    }
    // MYTHGPU_JIT_ASM_GEN_ONLY=1 (diagnostic, search kernels): only the generator — every coordinate
    // generated whole, nothing else evaluated (verdict 1): the generator's share of the kernel's VALU
    if (gen_only() && !eval_kernel) {
      std::vector<Instr> g;
      for (const Instr& in : code)
        if (in.op == K_COORD) g.push_back(in);
      code.swap(g);
      def.assign(P.vwidth.size(), -1);
      for (size_t k = 0; k < code.size(); k++) def[code[k].dst] = (int32_t)k;
      copysrc.assign(code.size(), MG_NONE);
      last.assign(P.vwidth.size(), -1);
      for (const Instr& in : code) need[in.dst] = lowmask(L(in.dst));
    }
    for (size_t kk = code.size(); kk-- > 0;) {
      const Instr& in = code[kk];
      const uint32_t d = in.dst;
      const uint64_t nd = (d != MG_NONE && d < need.size()) ? need[d] : 0;
      auto all = [&](uint32_t id) {
        if (id != MG_NONE && id < need.size()) need[id] |= lowmask(L(id));
      };
      auto upto = [&](uint32_t id, uint64_t m) {  // limbs 0 .. top demanded limb of m
        if (id == MG_NONE || id >= need.size() || !m) return;
        const uint32_t top = 63 - (uint32_t)__builtin_clzll(m);
        need[id] |= lowmask(top + 1) & lowmask(L(id));
      };
      auto same = [&](uint32_t id, uint64_t m) {
        if (id != MG_NONE && id < need.size()) need[id] |= m & lowmask(L(id));
      };
      if (in.op == K_COORD && copysrc[kk] != MG_NONE) all(copysrc[kk]);  // copied whole
      switch (in.op) {
        case K_ASSERT: all(in.a); break;
        case K_WATCH: if (eval_kernel) all(in.a); break;
        case K_ADD: case K_SUB: case K_MUL: upto(in.a, nd); upto(in.b, nd); break;
        case K_UDIV: case K_UREM: case K_SDIV: case K_SREM: case K_SMOD: case K_SHL: case K_LSHR: case K_ASHR:
        case K_EXP:
          if (nd) {
            all(in.a);
            all(in.b);
          }
          break;
        case K_KECCAK: if (nd && in.a != MG_NONE) all(in.a); break;
        case K_UMUL_NOOVF: all(in.a); all(in.b); break;
        case K_NEG: upto(in.a, nd); break;
        case K_AND: case K_OR: case K_XOR: same(in.a, nd); same(in.b, nd); break;
        case K_NOT: case K_COPY: same(in.a, nd); break;
        case K_ITE: all(in.a); same(in.b, nd); same(in.c, nd); break;
        case K_EQ: case K_ULT: case K_ULE: case K_SLT: case K_SLE: all(in.a); all(in.b); break;
        case K_ZEXT: same(in.a, nd); break;
        case K_SEXT: {
          const uint32_t La = Lw(in.p1);
          same(in.a, nd);
          if (nd >> (La - 1)) need[in.a] |= 1ull << (La - 1);
          break;
        }
        case K_EXTRACT:
          for (uint32_t j = 0; j < 64; j++)
            if (nd >> j & 1) need[in.a] |= bit_limbs(in.p0 + 32 * j, 32, in.p1);
          break;
        case K_CONCAT: {
          const uint32_t wb = in.p1, W = in.wd;
          for (uint32_t j = 0; j < 64; j++) {
            if (!(nd >> j & 1)) continue;
            const uint32_t p = 32 * j, e = std::min(W, p + 32);
            if (p < wb) need[in.b] |= bit_limbs(p, std::min(e, wb) - p, wb);
            if (e > wb) {
              const uint32_t q = std::max(p, wb) - wb;
              need[in.a] |= bit_limbs(q, e - std::max(p, wb), W - wb);
            }
          }
          break;
        }
        case K_LOOKUP:
          all(in.a);
          same(in.p0, nd);
          for (uint32_t q = 0; q < in.c; q++) {
            all(P.vaux[in.p1 + 2 * q]);
            same(P.vaux[in.p1 + 2 * q + 1], nd);
          }
          break;
        default: break;
      }
    }
    plan_views();
  }

  // Views: a CONCAT / EXTRACT / ZEXT value whose one reader is a CONCAT or an EXTRACT is never
  // materialised — its reader takes the bits it needs from the view's operands (field()).  A chain
  // of byte CONCATs building a word (calldata, storage keys) then costs a v_lshl_or per byte of the
  // word's low limb and aliases the rest, where materialising every link re-aligned every limb at
  // every link (C4's eval program: 1,565 VALU per candidate in CONCATs).  The view's operands live
  // until its reader (last[] extended).  MYTHGPU_JIT_ASM_NO_VIEWS=1 materialises every value.
  // K_MUL by operand pair (unordered) and width -> its vcode index: an UMUL_NOOVF of the same pair
  // before it computes the low limbs of the same product (mulshare)
  std::map<std::tuple<uint32_t, uint32_t, uint32_t>, size_t> mul_at;
  std::map<std::pair<uint32_t, uint32_t>, std::vector<Limb>> mulshare;  // owned limbs, until the MUL
  std::vector<uint8_t> view;  // value id -> a view
  std::vector<uint32_t> slt_lits;  // value id -> signed compares of it against a literal
  bool slt_many = false;           // the compare being emitted reads such a value 3+ times
  void plan_views() {
    const size_t nv = P.vwidth.size();
    view.assign(nv, 0);
    slt_lits.assign(nv, 0);
    mul_at.clear();
    for (size_t k = 0; k < code.size(); k++) {
      const Instr& in = code[k];
      if (in.op == K_MUL && !mul_at.count({std::min(in.a, in.b), std::max(in.a, in.b), in.wd}))
        mul_at[{std::min(in.a, in.b), std::max(in.a, in.b), in.wd}] = k;
    }
    for (const Instr& in : code) {
      if (in.op != K_SLT && in.op != K_SLE) continue;
      const Instr* da = def_of(in.a);
      const Instr* db = def_of(in.b);
      if (da && da->op == K_CONST && in.b < nv) slt_lits[in.b]++;
      if (db && db->op == K_CONST && in.a < nv) slt_lits[in.a]++;
    }
    static const bool off = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_VIEWS");
      return g && g[0] == '1';
    }();
    if (off) return;
    std::vector<uint32_t> nuse(nv, 0);
    std::vector<uint8_t> field_only(nv, 1);
    auto reader = [&](uint32_t id, uint32_t op) {
      if (id == MG_NONE || id >= nv) return;
      nuse[id]++;
      if (op != K_CONCAT && op != K_EXTRACT) field_only[id] = 0;
    };
    for (size_t k = 0; k < code.size(); k++) {
      const Instr& in = code[k];
      switch (in.op) {
        case K_CONST: break;
        case K_WATCH: if (eval_kernel) reader(in.a, in.op); break;
        case K_COORD: if (copysrc[k] != MG_NONE) reader(copysrc[k], in.op); break;
        case K_LOOKUP:
          reader(in.a, in.op);
          reader(in.p0, in.op);
          for (uint32_t q = 0; q < 2 * in.c; q++) reader(P.vaux[in.p1 + q], in.op);
          break;
        default:
          reader(in.a, in.op);
          if (in.op != K_NOT && in.op != K_NEG && in.op != K_EXTRACT && in.op != K_ZEXT && in.op != K_SEXT &&
              in.op != K_ASSERT && in.op != K_COPY)
            reader(in.b, in.op);
          if (in.op == K_ITE) reader(in.c, in.op);
          break;
      }
    }
    for (size_t k = code.size(); k-- > 0;) {  // readers before their operands: chains extend in one pass
      const Instr& in = code[k];
      const uint32_t d = in.dst;
      if (d == MG_NONE || d >= nv || def[d] != (int32_t)k) continue;
      if (in.op != K_CONCAT && in.op != K_EXTRACT && in.op != K_ZEXT) continue;
      if (in.wd <= 1 || nuse[d] != 1 || !field_only[d] || last[d] < 0) continue;
      view[d] = 1;
      for (uint32_t o : {in.a, in.op == K_CONCAT ? in.b : MG_NONE})
        if (o != MG_NONE && o < nv) last[o] = std::max(last[o], last[d]);
    }
  }
  bool is_view(uint32_t id) const { return id != MG_NONE && id < view.size() && view[id]; }

  void plan_lds() {
    // coordinates a search reads: the program's K_COORDs and, transitively, their COPY sources
    std::vector<char> reach(specs.size(), 0);
    std::vector<uint32_t> st;
    for (const Instr& in : code)
      if (in.op == K_COORD && in.p0 < reach.size() && !reach[in.p0]) {
        reach[in.p0] = 1;
        st.push_back(in.p0);
      }
    while (!st.empty()) {
      const uint32_t x = st.back();
      st.pop_back();
      const GenSpec& sp = specs[x];
      if ((sp.kind & 0xFFu) == MG_GEN_MIXED && sp.p[3] != MG_NONE && (sp.p[2] & 0xFFFFu) && sp.p[3] < reach.size() &&
          !reach[sp.p[3]]) {
        reach[sp.p[3]] = 1;
        st.push_back(sp.p[3]);
      }
    }
    for (uint32_t c = 0; c < specs.size() && c < P.coord_width.size(); c++) {
      if (!reach[c]) continue;
      const GenSpec& sp = specs[c];
      const uint32_t kind = sp.kind & 0xFFu, n = sp.p[1], off = sp.p[0], w = P.coord_width[c], Lc = Lw(w);
      const bool dict = kind == MG_GEN_DICT || (kind == MG_GEN_MIXED && n && (sp.p[2] >> 16));
      // small dictionaries too (the actor / sender addresses: 3 entries): a select chain is two VALU
      // per entry and limb, the LDS read none (its few addresses fall in distinct banks)
      if (!dict || n < 2 || Lc > 16 || lds_base.count(off)) continue;
      if (w <= 32 && (uint64_t)n * w <= 32) continue;  // packed into one literal
      // pair layout (lds_pairs): limbs (2p, 2p+1) of entry e side by side at word base + 2pn + 2e, an odd
      // top limb padded, the base even (8-byte aligned for ds_read_b64)
      const uint32_t Ls = lds_pairs() ? Lc + (Lc & 1u) : Lc, at = lds_pairs() ? (lds_words + 1u) & ~1u : lds_words;
      if ((size_t)off + (size_t)n * Lc > G.size() || at + n * Ls > kLdsWords) continue;
      lds_base[off] = at;
      lds_shape[off] = {n, Lc};
      lds_words = at + n * Ls;
    }
  }

  // prologue: every lane of the block copies words of the planned tables, then a barrier.  The loads
  // of up to stage_batch() (table, word) steps go out before one wait and their stores (a wait per step had
  // serialised one memory latency per table and step in every block's start-up: C3's first tier ran
  // 283 G/s at 64 blocks per CU and 424 at 32, profiles/r05p_rates_c3_bpc.jsonl)
  // MYTHGPU_JIT_ASM_STAGE_BATCH: steps per wait (default 1 until measured on the box; 16 batched)
  // Staged dictionaries in pairs of limbs, read by ds_read_b64: 8 bytes per lane in the LDS cycles and
  // lane groups a ds_read_b32 moves 4 in (64 banks instead of 32), so a lookup costs half the LDS
  // array cycles, bank conflicts included.  MYTHGPU_JIT_ASM_LDS_B32=1: one limb per read (limb-major)
  static bool lds_pairs() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_LDS_B32");
      return !(g && g[0] == '1');
    }();
    return on;
  }
  static size_t stage_batch() {
    static const size_t n = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_STAGE_BATCH");
      return g ? (size_t)std::max(1, std::min(32, atoi(g))) : (size_t)1;
    }();
    return n;
  }
  void emit_lds_prologue() {
    if (!lds_words) return;
    std::vector<std::pair<Limb, Limb>> pend;  // (loaded word, LDS address)
    auto flush = [&]() {
      if (pend.empty()) return;
      E.ctl("s_waitcnt vmcnt(0)");
      for (auto& pr : pend) {
        E.mem("ds_write_b32 " + VL(pr.second) + ", " + VL(pr.first));
        drop(pr.first);
        drop(pr.second);
      }
      pend.clear();
    };
    for (const auto& kv : lds_base) {
      const uint32_t off = kv.first, base = kv.second, n = lds_shape[off].first, Lc = lds_shape[off].second;
      const uint32_t nL = n * Lc, M = (65536u + Lc - 1) / Lc;  // i / Lc = (i * M) >> 16 for i * Lc < 2^16
      for (uint32_t it = 0; it * 256 < nL; it++) {
        const Limb vi = fresh(), vt = fresh(), ve = fresh(), vj = fresh();
        // word i = tid + 256 it, clamped to the last word (lanes past the table rewrite that one)
        E.valu("v_add_u32_e32 " + VL(vi) + ", " + imm(256 * it) + ", v0");
        E.valu("v_min_u32_e32 " + VL(vi) + ", " + imm(nL - 1) + ", " + VL(vi));
        E.valu("v_lshlrev_b32_e32 " + VL(vt) + ", 2, " + VL(vi));
        if (off * 4 < 4096) {
          E.mem("global_load_dword " + VL(vt) + ", " + VL(vt) + ", s[4:5] offset:" + std::to_string(off * 4));
        } else {
          E.valu("v_add_u32_e32 " + VL(vt) + ", " + hexs(off * 4) + ", " + VL(vt));
          E.mem("global_load_dword " + VL(vt) + ", " + VL(vt) + ", s[4:5]");
        }
        E.valu("v_mul_u32_u24_e32 " + VL(ve) + ", " + imm(M) + ", " + VL(vi));
        E.valu("v_lshrrev_b32_e32 " + VL(ve) + ", 16, " + VL(ve));       // entry e
        E.valu("v_mul_u32_u24_e32 " + VL(vj) + ", " + imm(Lc) + ", " + VL(ve));
        E.valu("v_sub_u32_e32 " + VL(vj) + ", " + VL(vi) + ", " + VL(vj));  // limb j
        if (lds_pairs()) {  // word base + (j & ~1) n + 2e + (j & 1)
          const Limb vo = fresh();
          E.valu("v_and_b32_e32 " + VL(vo) + ", 1, " + VL(vj));
          E.valu("v_and_b32_e32 " + VL(vj) + ", -2, " + VL(vj));
          E.valu("v_mul_u32_u24_e32 " + VL(vj) + ", " + imm(n) + ", " + VL(vj));
          E.valu("v_lshl_add_u32 " + VL(ve) + ", " + VL(ve) + ", 1, " + VL(vo));
          drop(vo);
        } else {
          E.valu("v_mul_u32_u24_e32 " + VL(vj) + ", " + imm(n) + ", " + VL(vj));
        }
        if (!inl(base)) E.salu("s_mov_b32 s41, " + hexs(base), {41});
        E.valu("v_add3_u32 " + VL(vj) + ", " + VL(vj) + ", " + VL(ve) + ", " + (inl(base) ? imm(base) : "s41"), {41});
        E.valu("v_lshlrev_b32_e32 " + VL(vj) + ", 2, " + VL(vj));
        drop(vi);
        drop(ve);
        pend.push_back({vt, vj});
        if (pend.size() >= stage_batch()) flush();
      }
    }
    flush();
    E.ctl("s_waitcnt lgkmcnt(0)");
    E.ctl("s_barrier");
  }

  // ---------------------------------------------------------------------------------------
  // operand helpers
  // ---------------------------------------------------------------------------------------
  Emitter& e() { return E; }

  // Code emitted under a condition (a MIXED alternative, a delta step, a division / EXP / Keccak
  // loop) may not run on every path to a later use, so nothing computed there enters the value
  // caches (xcache, litcache): cond counts the open conditional regions
  int cond = 0;
  struct CondScope {
    Gen& g;
    explicit CondScope(Gen& g_) : g(g_) { g.cond++; }
    ~CondScope() { g.cond--; }
  };
  // literals materialised in VGPRs, reused while the current constraint's code is emitted (cleared at
  // each ASSERT and under register pressure): a LOOKUP's select chain over a literal default or
  // literal-tail keys moved the same literal into a VGPR once per limb and prior
  std::map<uint32_t, Limb> litcache;  // each entry holds one reference
  // last use of each cache entry (eviction under the soft VGPR limit: least recently used first)
  uint64_t tick = 0;
  std::map<uint32_t, uint64_t> lit_last;
  std::map<std::pair<uint64_t, uint64_t>, uint64_t> x_last;
  std::map<std::pair<uint32_t, uint32_t>, uint64_t> eq_last;
  void litcache_clear() {
    std::vector<Limb> held;
    for (auto& kv : litcache) held.push_back(kv.second);
    litcache.clear();
    lit_last.clear();
    for (auto& d : held) drop(d);
  }
  // a VGPR holding limb l (a literal is moved into a fresh VGPR the caller releases)
  Limb vreg(const Limb& l) {
    if (l.reg()) {
      E.retain(l);
      return l;
    }
    const uint32_t x = l.lit() ? l.v : 0u;
    if (x == 0) return Reg(6);  // the zero register
    auto it = pool.find(x);
    if (it != pool.end()) return Reg((uint32_t)it->second);  // loaded once, before the group loop
    const bool cache = !cond && !no_lvn() && lvn_on && caches;
    if (cache) {
      auto c = litcache.find(x);
      if (c != litcache.end()) {
        lit_last[x] = ++tick;
        E.retain(c->second);
        return c->second;
      }
    }
    census[x]++;
    const Limb r = fresh();
    E.valu("v_mov_b32_e32 " + VL(r) + ", " + imm(x));
    if (cache) {
      E.retain(r);
      litcache[x] = r;
      lit_last[x] = ++tick;
    }
    return r;
  }
  bool lvn_on = false;  // the value caches are live only inside body()
  // jit_asm_source's first pass emits without the value caches (litcache, xcache, eqdiff): its VGPR
  // count sets the occupancy step (vsoft) the cached second pass must stay within
  bool caches = true;
  int vsoft = 256;
  // Literal pool: literals a VGPR operand needs (select arms, carry-chain operands, dictionary
  // entries) are moved into a VGPR at every use unless pooled — one VGPR each, loaded once per
  // kernel before the group loop.  jit_asm_source emits twice: the first pass counts (census), the
  // second pools the most used ones within the VGPR budget.
  std::map<uint32_t, int> pool;        // literal -> its VGPR
  std::map<uint32_t, uint32_t> census; // literal -> materialisations in the last emission
  std::string src(const Limb& l) const {
    if (l.k == LU) fail("internal: a limb the demand analysis dropped was read");
    E.check(l);
    return l.lit() ? imm(l.v) : VL(l);
  }

  // operand usable in a VOP3 slot: VGPR or inline constant (other literals go through a VGPR)
  Limb v3(const Limb& l) {
    if (l.lit() && inl(l.v)) return l;
    return vreg(l);
  }
  void drop(const Limb& l) { E.release(l); }

  Limb fresh() {
    const uint32_t r = E.valloc();
    return Limb{LR, r, E.vgen[r]};
  }
  // x * y (x a VGPR, y a VGPR or an operand string `so`: an inline constant or s41) as (lo, hi): one
  // v_mad_u64_u32 into a register pair when both halves are wanted — one instruction for what
  // v_mul_lo_u32 + v_mul_hi_u32 take two (LLVM's choice for the O3 kernels' products too);
  // MYTHGPU_JIT_ASM_NO_MAD=1: the two multiplies
  static bool no_mad() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_MAD");
      return g && g[0] == '1';
    }();
    return on;
  }
  void product(const Limb& vx, const std::string& so, bool s41, bool want_lo, bool want_hi, Limb& lo, Limb& hi) {
    std::initializer_list<int> none{};
    if (want_lo && want_hi && !no_mad()) {
      const uint32_t r = E.valloc2();
      lo = Limb{LR, r, E.vgen[r]};
      hi = Limb{LR, r + 1, E.vgen[r + 1]};
      Mask c;  // the carry-out pair the encoding names (always 0: the addend is 0)
      c.k = 2;
      c.s = E.salloc();
      const std::string ins = "v_mad_u64_u32 v[" + std::to_string(r) + ":" + std::to_string(r + 1) + "], " + SP(c.s) +
                              ", " + VL(vx) + ", " + so + ", 0";
      if (s41) E.valu(ins, {41}, {c.s, c.s + 1});
      else E.valu(ins, none, {c.s, c.s + 1});
      E.srelease(c);
      return;
    }
    if (want_lo) {
      lo = fresh();
      if (s41) E.valu("v_mul_lo_u32 " + VL(lo) + ", " + VL(vx) + ", " + so, {41});
      else E.valu("v_mul_lo_u32 " + VL(lo) + ", " + VL(vx) + ", " + so);
    }
    if (want_hi) {
      hi = fresh();
      if (s41) E.valu("v_mul_hi_u32 " + VL(hi) + ", " + VL(vx) + ", " + so, {41});
      else E.valu("v_mul_hi_u32 " + VL(hi) + ", " + VL(vx) + ", " + so);
    }
  }
  // the register name of a limb, checked against its allocation (MYTHGPU_JIT_ASM_CHECK)
  std::string VL(const Limb& l) const {
    E.check(l);
    if (!E.lds_pending.empty() && l.reg() && E.lds_pending.count((int)l.v)) E.lds_flush();
    return V(l.v);
  }

  // mask form of a Bool value
  Mask mask_of(uint32_t id) {
    Val& x = val[id];
    if (x.m.k) return x.m;
    const Limb l = x.l.empty() ? Lit(0) : x.l[0];
    Mask m;
    if (l.lit() || l.k == LU) {
      m.k = 1;
      m.ones = l.lit() && (l.v & 1u);
    } else {
      m.k = 2;
      m.s = E.salloc();
      E.valu("v_cmp_ne_u32_e64 " + SP(m.s) + ", 0, " + VL(l), {}, {m.s, m.s + 1});
    }
    x.m = m;
    return m;
  }
  // limb form of a Bool value
  Limb limb_of_bool(uint32_t id) {
    Val& x = val[id];
    if (!x.l.empty() && x.l[0].k != LU) return x.l[0];
    const Mask m = mask_of(id);
    Limb l;
    if (m.k == 1) {
      l = Lit(m.ones ? 1u : 0u);
    } else {
      l = fresh();
      E.valu("v_cndmask_b32_e64 " + VL(l) + ", 0, 1, " + SP(m.s), {m.s, m.s + 1});
    }
    x.l.assign(1, l);
    return l;
  }
  // limb j of value id (Bools through their limb form)
  Limb limb(uint32_t id, uint32_t j) {
    if (P.vwidth[id] == 1 && j == 0) return limb_of_bool(id);
    if (is_spilled(id)) reload(id);
    const Val& x = val[id];
    if (j >= x.l.size()) return Lit(0);
    return x.l[j];
  }
  bool is_bool(uint32_t id) const { return P.vwidth[id] == 1; }

  // ---------------------------------------------------------------------------------------
  // limb arithmetic
  // ---------------------------------------------------------------------------------------
  // x + y (+ carry) over limbs lo..hi of the result; `carry` -1: in VCC, 0/1 known
  // returns the result limbs; the carry out ends in VCC (or known)
  std::vector<Limb> add_chain(const std::vector<Limb>& x, const std::vector<Limb>& y, uint32_t n, bool sub) {
    std::vector<Limb> r(n);
    int carry = 0;  // known 0/1, or -1 = VCC
    Limb zz{};      // a subtraction's 0 - 0 - borrow limb (the same for every such limb above)
    for (uint32_t j = 0; j < n; j++) {
      const Limb a = j < x.size() ? x[j] : Lit(0), b = j < y.size() ? y[j] : Lit(0);
      if (carry < 0 && a.lit() && a.v == 0 && b.lit() && b.v == 0) {
        // zero limbs above a carry in VCC: an addition's limb is the carry and carries nothing on (the
        // limbs above are literal zeros); a subtraction's is -borrow, borrowing on — one limb serves all
        if (!sub) {
          const Limb d = fresh();
          E.valu("v_addc_co_u32_e32 " + VL(d) + ", vcc, 0, v6, vcc", {kVCC, kVCC + 1}, {kVCC, kVCC + 1});
          r[j] = d;
          carry = 0;
          continue;
        }
        if (!zz.reg()) {
          zz = fresh();
          E.valu("v_subb_co_u32_e32 " + VL(zz) + ", vcc, 0, v6, vcc", {kVCC, kVCC + 1}, {kVCC, kVCC + 1});
          r[j] = zz;
        } else {
          E.retain(zz);
          r[j] = zz;
        }
        continue;
      }
      zz = Limb{};  // a different borrow from here on
      if (a.lit() && b.lit() && carry >= 0) {
        uint64_t t;
        if (!sub) {
          t = (uint64_t)a.v + b.v + (uint64_t)carry;
          carry = (int)(t >> 32);
        } else {
          t = (uint64_t)a.v - b.v - (uint64_t)carry;
          carry = ((uint64_t)a.v < (uint64_t)b.v + (uint64_t)carry) ? 1 : 0;
        }
        r[j] = Lit((uint32_t)t);
        continue;
      }
      if (carry == 0 && ((!sub && a.lit() && a.v == 0) || (b.lit() && b.v == 0))) {
        r[j] = (b.lit() && b.v == 0) ? a : b;  // x + 0, 0 + y, x - 0: no carry
        E.retain(r[j]);
        continue;
      }
      if (carry == 1) {
        E.salu("s_mov_b64 vcc, -1", {kVCC, kVCC + 1});
        carry = -1;
      }
      const Limb d = fresh();
      if (carry == 0) {
        if (!sub) {
          const Limb s0 = b.reg() ? a : b, s1 = b.reg() ? b : a;  // src1 must be a VGPR
          E.valu("v_add_co_u32_e32 " + VL(d) + ", vcc, " + src(s0) + ", " + VL(s1), {}, {kVCC, kVCC + 1});
        } else if (b.reg()) {
          E.valu("v_sub_co_u32_e32 " + VL(d) + ", vcc, " + src(a) + ", " + VL(b), {}, {kVCC, kVCC + 1});
        } else {
          E.valu("v_subrev_co_u32_e32 " + VL(d) + ", vcc, " + src(b) + ", " + VL(a), {}, {kVCC, kVCC + 1});
        }
      } else {
        Limb aa = a, bb = b, tmp, tmp2;
        if (!aa.reg() && !bb.reg()) {
          if (bb.lit() && bb.v == 0) bb = Reg(6);  // the zero register
          else if (!sub && aa.lit() && aa.v == 0) aa = Reg(6);
          else {
            tmp = vreg(bb);
            bb = tmp;
          }
        }
        // the carry-in (VCC) is on the constant bus: the other operand must not be a literal
        if (aa.lit() && !inl(aa.v)) {
          tmp2 = vreg(aa);
          aa = tmp2;
        } else if (bb.lit() && !inl(bb.v)) {
          tmp2 = vreg(bb);
          bb = tmp2;
        }
        if (!sub) {
          const Limb s0 = bb.reg() ? aa : bb, s1 = bb.reg() ? bb : aa;
          E.valu("v_addc_co_u32_e32 " + VL(d) + ", vcc, " + src(s0) + ", " + VL(s1) + ", vcc", {kVCC, kVCC + 1},
                 {kVCC, kVCC + 1});
        } else if (bb.reg()) {
          E.valu("v_subb_co_u32_e32 " + VL(d) + ", vcc, " + src(aa) + ", " + VL(bb) + ", vcc", {kVCC, kVCC + 1},
                 {kVCC, kVCC + 1});
        } else {
          E.valu("v_subbrev_co_u32_e32 " + VL(d) + ", vcc, " + src(bb) + ", " + VL(aa) + ", vcc", {kVCC, kVCC + 1},
                 {kVCC, kVCC + 1});
        }
        drop(tmp);
        drop(tmp2);
      }
      carry = -1;
      r[j] = d;
    }
    last_carry = carry;
    return r;
  }
  int last_carry = 0;

  // d = x & m (m literal): folded, or one v_and_b32
  Limb and_lit(const Limb& x, uint32_t m) {
    if (x.lit()) return Lit(x.v & m);
    if (m == 0) return Lit(0);
    if (m == 0xFFFFFFFFu) {
      E.retain(x);
      return x;
    }
    const Limb d = fresh();
    E.valu("v_and_b32_e32 " + VL(d) + ", " + imm(m) + ", " + VL(x));
    return d;
  }
  // the top limb of a width-w result masked (the limb vector owns its registers)
  void mask_top(std::vector<Limb>& r, uint32_t w) {
    if (!(w & 31) || r.empty()) return;
    Limb& t = r.back();
    if (t.k == LU) return;
    const Limb m = and_lit(t, topmask(w));
    drop(t);
    t = m;
  }

  // bits [p, p+n) (n <= 32) of the limb vector x (width w) at bit 0, zero above n
  Limb bits(const std::vector<Limb>& x, uint32_t w, uint32_t p, uint32_t n) {
    if (p >= w || n == 0) return Lit(0);
    n = std::min(n, w - p);
    const uint32_t q = p / 32, r = p % 32;
    const Limb lo = q < x.size() ? x[q] : Lit(0);
    const bool need_hi = r && r + n > 32 && (q + 1) * 32 < w;
    const Limb hi = need_hi && q + 1 < x.size() ? x[q + 1] : Lit(0);
    const bool clip = n < 32 && p + n < w;  // bits above n may be set
    const uint32_t m = n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u);
    if (lo.k == LU || (need_hi && hi.k == LU)) fail("internal: a limb the demand analysis dropped was read");
    if (!need_hi || (hi.lit() && hi.v == 0 && !r)) {
      if (r == 0) {
        if (!clip) {
          E.retain(lo);
          return lo;
        }
        return and_lit(lo, m);
      }
      if (lo.lit()) return Lit((lo.v >> r) & (clip ? m : 0xFFFFFFFFu));
      const Limb d = fresh();
      if (clip) E.valu("v_bfe_u32 " + VL(d) + ", " + VL(lo) + ", " + std::to_string(r) + ", " + std::to_string(n));
      else E.valu("v_lshrrev_b32_e32 " + VL(d) + ", " + std::to_string(r) + ", " + VL(lo));
      return d;
    }
    if (lo.lit() && hi.lit()) {
      const uint32_t t = (uint32_t)((((uint64_t)hi.v << 32) | lo.v) >> r);
      return Lit(clip ? (t & m) : t);
    }
    const Limb a = v3(hi), b = v3(lo);
    const Limb d = fresh();
    E.valu("v_alignbit_b32 " + VL(d) + ", " + src(a) + ", " + src(b) + ", " + std::to_string(r));
    drop(a);
    drop(b);
    if (!clip) return d;
    const Limb c = and_lit(d, m);
    drop(d);
    return c;
  }

  // bits [p, p+n) (n <= 32) of value id at bit 0, zero above n (owned): through views (plan_views)
  // to the materialised limbs they are made of
  Limb field(uint32_t id, uint32_t p, uint32_t n) {
    const uint32_t w = P.vwidth[id];
    if (p >= w || n == 0) return Lit(0);
    n = std::min(n, w - p);
    if (!is_view(id)) return bits(limbs(id, Lw(w)), w, p, n);
    return field_of(code[def[id]], p, n);
  }
  // the same of the value instruction `in` (a CONCAT, EXTRACT or ZEXT) defines
  Limb field_of(const Instr& in, uint32_t p, uint32_t n) {
    switch (in.op) {
      case K_EXTRACT: return field(in.a, in.p0 + p, n);
      case K_ZEXT: return field(in.a, p, n);  // bits above the operand: zero
      case K_CONCAT: {  // a (high) : b (low, p1 bits)
        const uint32_t wb = in.p1;
        if (p + n <= wb) return field(in.b, p, n);
        if (p >= wb) return field(in.a, p - wb, n);
        const Limb lo = field(in.b, p, wb - p), hi = field(in.a, 0, p + n - wb);
        const Limb r = shl_or(hi, wb - p, lo);
        drop(lo);
        drop(hi);
        return r;
      }
      default: fail("internal: a view of op " + std::to_string(in.op));
    }
    return Lit(0);
  }

  // (hi << s) | lo, lo < 2^s
  Limb shl_or(const Limb& hi, uint32_t s, const Limb& lo) {
    if (hi.lit() && lo.lit()) return Lit((s < 32 ? hi.v << s : 0u) | lo.v);
    if (hi.lit() && hi.v == 0) {
      E.retain(lo);
      return lo;
    }
    const Limb a = v3(hi), c = v3(lo);
    const Limb d = fresh();
    E.valu("v_lshl_or_b32 " + VL(d) + ", " + src(a) + ", " + std::to_string(s) + ", " + src(c));
    drop(a);
    drop(c);
    return d;
  }

  // XOR-OR reduction of the limb pairs -> mask (all lanes where every pair is equal).  Pairs whose XOR
  // the limb cache holds (xcache) are ORed in; the others accumulate one v_bitop3 each,
  // acc = (a ^ b) | acc (a literal operand through s41), instead of an XOR each and an OR tree
  // (MYTHGPU_JIT_ASM_EQ_BITOP3=0: XOR each pair, then OR3 trees)
  static bool eq_bitop3() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_EQ_BITOP3");
      return !(g && g[0] == '0');
    }();
    return on;
  }
  // Dictionary limbs: a register that holds limb j of entry `idx` of a pure DICT coordinate's table
  // (gen_value), keyed by its allocation tag, with the entry index register (one reference each).
  // A compare of such limbs with literals, or with the same limbs of another coordinate drawn from an
  // equal table, is decided by the indices: C4's key tests of caller-keyed mappings (the caller
  // against the three actor literals) cost one compare of the index instead of an XOR-OR reduction
  // over five limbs — what LLVM finds in the O3 kernel from its select chains.
  // MYTHGPU_JIT_ASM_NO_DICT_EQ=1: off
  struct DLimb {
    uint32_t off = 0, n = 0, Lc = 0, j = 0;
    Limb idx;
  };
  std::map<uint32_t, DLimb> dlimb;
  static bool no_dict_eq() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_DICT_EQ");
      return g && g[0] == '1';
    }();
    return on;
  }
  void dlimb_free(uint32_t g) {
    auto it = dlimb.find(g);
    if (it == dlimb.end()) return;
    const Limb ix = it->second.idx;
    dlimb.erase(it);
    drop(ix);
  }
  bool dict_limb(const Limb& l, DLimb& out) const {
    if (!l.reg() || !l.g || (int)l.v < E.vfirst || E.vgen[l.v] != l.g) return false;
    auto it = dlimb.find(l.g);
    if (it == dlimb.end()) return false;
    out = it->second;
    return true;
  }
  // the lane mask of idx in the entry set S (bit e), n entries; false when it takes more than two VALU
  bool idx_in_set(const Limb& idx, const std::vector<char>& S, uint32_t n, Mask& m) {
    uint32_t cnt = 0, first = 0, miss = 0;
    for (uint32_t e = 0; e < n; e++) {
      if (S[e]) {
        if (!cnt) first = e;
        cnt++;
      } else {
        miss = e;
      }
    }
    if (cnt == 0 || cnt == n) {
      m.k = 1;
      m.ones = cnt == n;
      return true;
    }
    if (cnt != 1 && cnt != n - 1 && n > 32) return false;
    m.k = 2;
    m.s = E.salloc();
    if (cnt == 1 || cnt == n - 1) {
      const uint32_t e = cnt == 1 ? first : miss;
      const std::string op = cnt == 1 ? "v_cmp_eq_u32" : "v_cmp_ne_u32";
      if (inl(e)) {
        E.valu(op + "_e64 " + SP(m.s) + ", " + imm(e) + ", " + VL(idx), {}, {m.s, m.s + 1});
      } else {
        E.valu(op + "_e32 vcc, " + hexs(e) + ", " + VL(idx), {}, {kVCC, kVCC + 1});
        E.salu("s_mov_b64 " + SP(m.s) + ", vcc", {m.s, m.s + 1});
      }
      return true;
    }
    uint32_t bits = 0;
    for (uint32_t e = 0; e < n; e++)
      if (S[e]) bits |= 1u << e;
    const Limb t = fresh();
    E.salu("s_mov_b32 s41, " + hexs(bits), {41});
    E.valu("v_bfe_u32 " + VL(t) + ", s41, " + VL(idx) + ", 1", {41});
    E.valu("v_cmp_ne_u32_e64 " + SP(m.s) + ", 0, " + VL(t), {}, {m.s, m.s + 1});
    drop(t);
    return true;
  }
  // a == b over limb pairs decided by dictionary indices (above); false: the general reduction
  bool dict_eq(const std::vector<std::pair<Limb, Limb>>& prs, Mask& m) {
    if (no_dict_eq() || dlimb.empty()) return false;
    bool haveA = false, haveB = false;
    DLimb A, B;
    std::vector<std::pair<uint32_t, uint32_t>> lits;  // (limb of A, literal)
    std::vector<std::pair<uint32_t, uint32_t>> regs;  // (limb of A, limb of B)
    auto same_src = [](const DLimb& x, const DLimb& y) {
      return x.off == y.off && x.n == y.n && x.Lc == y.Lc && x.idx == y.idx && x.idx.g == y.idx.g;
    };
    for (const auto& pr : prs) {
      const Limb a = pr.first, b = pr.second;
      if (a.lit() && b.lit()) {
        if (a.v != b.v) {
          m.k = 1;
          m.ones = false;
          return true;
        }
        continue;
      }
      if (a == b) continue;
      DLimb da, db;
      const bool ia = dict_limb(a, da), ib = dict_limb(b, db);
      if ((ia && b.lit()) || (ib && a.lit())) {
        const DLimb& d = ia ? da : db;
        if (!haveA) {
          A = d;
          haveA = true;
        } else if (!same_src(A, d)) {
          return false;
        }
        lits.push_back({d.j, ia ? b.v : a.v});
      } else if (ia && ib) {
        if (!haveA) {
          A = da;
          haveA = true;
        }
        if (!haveB) {
          B = db;
          haveB = true;
        }
        const bool fwd = same_src(A, da) && same_src(B, db), rev = same_src(A, db) && same_src(B, da);
        if (!fwd && !rev) return false;
        const DLimb& x = fwd ? da : db;
        const DLimb& y = fwd ? db : da;
        regs.push_back({x.j, y.j});
      } else {
        return false;
      }
    }
    if (!haveA) return false;  // (only literal pairs: the general path folds them)
    if (!lits.empty() && !regs.empty()) return false;
    if (!lits.empty()) {
      std::vector<char> S(A.n, 0);
      for (uint32_t e = 0; e < A.n; e++) {
        bool ok = true;
        for (const auto& lj : lits) ok = ok && G[A.off + e * A.Lc + lj.first] == lj.second;
        S[e] = ok;
      }
      return idx_in_set(A.idx, S, A.n, m);
    }
    // two coordinates' entries: equal exactly when their indices are, if entry e of A matches entry e
    // of B and no other on the compared limbs
    if (!haveB || A.n != B.n || A.n > 256) return false;
    for (uint32_t e = 0; e < A.n; e++)
      for (uint32_t f = 0; f < B.n; f++) {
        bool eq = true;
        for (const auto& jj : regs) eq = eq && G[A.off + e * A.Lc + jj.first] == G[B.off + f * B.Lc + jj.second];
        if (eq != (e == f)) return false;
      }
    m.k = 2;
    m.s = E.salloc();
    E.valu("v_cmp_eq_u32_e64 " + SP(m.s) + ", " + VL(A.idx) + ", " + VL(B.idx), {}, {m.s, m.s + 1});
    return true;
  }
  Mask eq_mask(const std::vector<std::pair<Limb, Limb>>& prs, Limb* keep = nullptr) {
    {
      Mask dm;
      if (dict_eq(prs, dm)) return dm;
    }
    std::vector<Limb> diff;  // owned
    std::vector<std::pair<Limb, Limb>> raw;  // pairs for the bitop3 accumulation
    for (const auto& pr : prs) {
      const Limb a = pr.first, b = pr.second;
      if (a.lit() && b.lit()) {
        if (a.v != b.v) {
          for (auto& d : diff) drop(d);
          Mask m;
          m.k = 1;
          m.ones = false;
          return m;
        }
        continue;
      }
      if (a == b) continue;
      if (a.lit() && a.v == 0) {
        E.retain(b);
        diff.push_back(b);
        continue;
      }
      if (b.lit() && b.v == 0) {
        E.retain(a);
        diff.push_back(a);
        continue;
      }
      if (prs.size() == 1 || (diff.empty() && raw.empty() && &pr == &prs.back())) {
        // one pair only: one compare
        const Limb s0 = b.reg() ? a : b, s1 = b.reg() ? b : a;
        Mask m;
        m.k = 2;
        m.s = E.salloc();
        if (s0.lit() && !inl(s0.v)) {
          E.valu("v_cmp_eq_u32_e32 vcc, " + src(s0) + ", " + VL(s1), {}, {kVCC, kVCC + 1});
          E.salu("s_mov_b64 " + SP(m.s) + ", vcc", {m.s, m.s + 1});
        } else {
          E.valu("v_cmp_eq_u32_e64 " + SP(m.s) + ", " + src(s0) + ", " + VL(s1), {}, {m.s, m.s + 1});
        }
        return m;
      }
      if (eq_bitop3()) {
        Limb hit;
        if (xcache_get(a, b, hit)) diff.push_back(hit);
        else raw.push_back({a, b});
      } else {
        diff.push_back(xor_limb(a, b));
      }
    }
    if (!raw.empty()) {
      // acc = a0 ^ b0, then acc = (a ^ b) | acc per pair (bitop3 table 0xBE over (a, b, acc))
      const auto& p0 = raw[0];
      Limb acc = fresh();
      {
        const Limb s0 = p0.second.reg() ? p0.first : p0.second, s1 = p0.second.reg() ? p0.second : p0.first;
        E.valu("v_xor_b32_e32 " + VL(acc) + ", " + src(s0) + ", " + VL(s1));
      }
      int64_t s41 = -1;  // the literal s41 holds
      for (size_t i = 1; i < raw.size(); i++) {
        const Limb x = raw[i].second.reg() ? raw[i].first : raw[i].second;  // a literal, if any
        const Limb y = raw[i].second.reg() ? raw[i].second : raw[i].first;
        std::string xs;
        if (x.lit() && !inl(x.v)) {
          if (s41 != (int64_t)x.v) {
            E.salu("s_mov_b32 s41, " + hexs(x.v), {41});
            s41 = x.v;
          }
          xs = "s41";
        } else {
          xs = src(x);
        }
        const Limb d = fresh();
        if (xs == "s41") E.valu("v_bitop3_b32 " + VL(d) + ", " + VL(y) + ", s41, " + VL(acc) + " bitop3:0xbe", {41});
        else E.valu("v_bitop3_b32 " + VL(d) + ", " + VL(y) + ", " + xs + ", " + VL(acc) + " bitop3:0xbe");
        drop(acc);
        acc = d;
      }
      diff.push_back(acc);
    }
    Mask m;
    if (diff.empty()) {
      m.k = 1;
      m.ones = true;
      return m;
    }
    while (diff.size() > 1) {
      std::vector<Limb> nx;
      for (size_t i = 0; i < diff.size(); i += 3) {
        const size_t k = std::min<size_t>(3, diff.size() - i);
        if (k == 1) {
          nx.push_back(diff[i]);
          continue;
        }
        const Limb d = fresh();
        if (k == 2) E.valu("v_or_b32_e32 " + VL(d) + ", " + VL(diff[i]) + ", " + VL(diff[i + 1]));
        else E.valu("v_or3_b32 " + VL(d) + ", " + VL(diff[i]) + ", " + VL(diff[i + 1]) + ", " + VL(diff[i + 2]));
        for (size_t t = 0; t < k; t++) drop(diff[i + t]);
        nx.push_back(d);
      }
      diff.swap(nx);
    }
    m.k = 2;
    m.s = E.salloc();
    E.valu("v_cmp_eq_u32_e64 " + SP(m.s) + ", 0, " + VL(diff[0]), {}, {m.s, m.s + 1});
    if (keep) *keep = diff[0];  // the caller holds the reduced difference (eq_ids' cache)
    else drop(diff[0]);
    return m;
  }

  // Limb value numbering of the compare differences: x ^ y of two limbs is kept while both limbs'
  // registers hold the values they had (allocation tags), so keys that share limbs across values —
  // Concat(sender, slot) vs Concat(sender, other slot), a COPY and its source, a key and the
  // LOOKUP priors built from it — XOR each limb pair once.  Each entry holds one reference to its
  // result; the entry goes when either operand's register is released for good (E.on_free).
  static uint64_t lid(const Limb& l) { return l.lit() ? ((1ull << 63) | l.v) : (((uint64_t)l.g << 9) | l.v); }
  std::map<std::pair<uint64_t, uint64_t>, Limb> xcache;
  std::multimap<uint32_t, std::pair<uint64_t, uint64_t>> xby;  // operand tag -> entries
  static bool no_lvn() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_LVN");
      return g && g[0] == '1';
    }();
    return on;
  }
  Limb xor_limb(const Limb& a, const Limb& b) {
    const Limb s0 = b.reg() ? a : b, s1 = b.reg() ? b : a;
    const bool cacheable = lvn_on && caches && !cond && !no_lvn() && (!s0.reg() || (int)s0.v < E.vfirst || s0.g) &&
                           ((int)s1.v < E.vfirst || s1.g);
    const uint64_t k0 = lid(s0), k1 = lid(s1);  // (std::minmax of temporaries would return dangling references)
    const std::pair<uint64_t, uint64_t> key(std::min(k0, k1), std::max(k0, k1));
    if (cacheable) {
      auto it = xcache.find(key);
      if (it != xcache.end()) {
        x_last[key] = ++tick;
        E.retain(it->second);
        return it->second;
      }
    }
    const Limb d = fresh();
    E.valu("v_xor_b32_e32 " + VL(d) + ", " + src(s0) + ", " + VL(s1));
    if (cacheable) {
      E.retain(d);
      xcache[key] = d;
      x_last[key] = ++tick;
      for (const Limb& o : {s0, s1})
        if (o.reg() && (int)o.v >= E.vfirst) xby.insert({o.g, key});
    }
    return d;
  }
  // the cached XOR of limbs a and b, if any (retained for the caller)
  bool xcache_get(const Limb& a, const Limb& b, Limb& out) {
    if (!(lvn_on && caches && !cond && !no_lvn())) return false;
    const uint64_t k0 = lid(a), k1 = lid(b);
    auto it = xcache.find({std::min(k0, k1), std::max(k0, k1)});
    if (it == xcache.end()) return false;
    x_last[it->first] = ++tick;
    E.retain(it->second);
    out = it->second;
    return true;
  }
  void xcache_free(uint32_t g) {
    auto r = xby.equal_range(g);
    std::vector<std::pair<uint64_t, uint64_t>> keys;
    for (auto it = r.first; it != r.second; ++it) keys.push_back(it->second);
    xby.erase(r.first, r.second);
    for (const auto& k : keys) {
      auto it = xcache.find(k);
      if (it == xcache.end()) continue;
      const Limb d = it->second;
      xcache.erase(it);
      drop(d);  // may free d's register in turn
    }
  }
  void xcache_clear() {
    std::vector<Limb> held;
    for (auto& kv : xcache) held.push_back(kv.second);
    xcache.clear();
    xby.clear();
    for (auto& d : held) drop(d);
    for (auto& kv : hcache) drop(kv.second);
    hcache.clear();
    hby.clear();
    h_last.clear();
  }
  // The reduced difference of a value's high limbs against a sign extension (slt_literal): LASER
  // compares one value with many literals (x >s 0, x >s 1, ... one per switch arm), whose high limbs
  // are the same registers each time — kept like the XOR cache, keyed by the limbs' allocation tags
  std::map<std::vector<uint64_t>, Limb> hcache;
  std::multimap<uint32_t, std::vector<uint64_t>> hby;
  std::map<std::vector<uint64_t>, uint64_t> h_last;
  void hcache_free(uint32_t g) {
    auto r = hby.equal_range(g);
    std::vector<std::vector<uint64_t>> keys;
    for (auto it = r.first; it != r.second; ++it) keys.push_back(it->second);
    hby.erase(r.first, r.second);
    for (const auto& k : keys) {
      auto it = hcache.find(k);
      if (it == hcache.end()) continue;
      const Limb d = it->second;
      hcache.erase(it);
      h_last.erase(k);
      drop(d);
    }
  }

  // a == b over the first Lk limbs of values a and b.  The reduced difference (OR of the limbs' XORs)
  // is kept while both values live: LASER's constraints compare the same keys again and again (a
  // keccak site's key against every prior site in each LOOKUP, and in the EQs of the injectivity
  // conditions), and a repeat then costs one compare
  std::map<std::pair<uint32_t, uint32_t>, Limb> eqdiff;  // each entry holds one reference
  Mask eq_ids(uint32_t a, uint32_t b, uint32_t Lk) {
    PinScope pin_(*this, {a, b});
    const auto key = std::minmax(a, b);
    auto it = eqdiff.find(key);
    if (it != eqdiff.end()) {
      eq_last[key] = ++tick;
      Mask m;
      m.k = 2;
      m.s = E.salloc();
      E.valu("v_cmp_eq_u32_e64 " + SP(m.s) + ", 0, " + VL(it->second), {}, {m.s, m.s + 1});
      return m;
    }
    std::vector<std::pair<Limb, Limb>> prs;
    for (uint32_t j = 0; j < Lk; j++) prs.push_back({limb(a, j), limb(b, j)});
    Limb keep{};
    const Mask m = eq_mask(prs, &keep);
    if (keep.reg() && caches) {
      eqdiff[key] = keep;
      eq_last[key] = ++tick;
    }
    else if (keep.reg()) drop(keep);
    return m;
  }
  // One cache entry goes, to make room under the soft VGPR limit: a literal first (a hit saves one
  // v_mov), then an XOR (one v_xor), then a compare difference (a whole OR-reduction), least
  // recently used first within each.  False when every cache is empty.
  template <class M, class T>
  static typename M::iterator lru(M& m, T& last) {
    auto best = m.end();
    uint64_t bt = ~0ull;
    for (auto it = m.begin(); it != m.end(); ++it) {
      auto l = last.find(it->first);
      const uint64_t t = l == last.end() ? 0 : l->second;
      if (t < bt) {
        bt = t;
        best = it;
      }
    }
    return best;
  }
  bool evict_one() {
    if (!litcache.empty()) {
      auto it = lru(litcache, lit_last);
      const Limb d = it->second;
      lit_last.erase(it->first);
      litcache.erase(it);
      drop(d);
      return true;
    }
    if (!xcache.empty()) {
      auto it = lru(xcache, x_last);
      const Limb d = it->second;
      x_last.erase(it->first);
      xcache.erase(it);  // its xby entries go stale: xcache_free skips keys no longer cached
      drop(d);
      return true;
    }
    if (!hcache.empty()) {
      auto it = lru(hcache, h_last);
      const Limb d = it->second;
      h_last.erase(it->first);
      hcache.erase(it);  // its hby entries go stale: hcache_free skips keys no longer cached
      drop(d);
      return true;
    }
    if (!eqdiff.empty()) {
      auto it = lru(eqdiff, eq_last);
      const Limb d = it->second;
      eq_last.erase(it->first);
      eqdiff.erase(it);
      drop(d);
      return true;
    }
    return false;
  }
  // Out of SGPR pairs (the compare pushdown keeps many Bools live as lane masks): the mask of the Bool
  // value read latest, and not by the instruction being emitted, moves to its VGPR form (one
  // v_cndmask; a later reader compares it back)
  size_t cur_k = 0;
  // MYTHGPU_JIT_ASM_ANNOTATE: a phase of the instruction being emitted, a tag of its own in the
  // simulator's per-tag counts (tools/asm_count.py)
  void note(const char* phase) {
    static const bool annotate = getenv("MYTHGPU_JIT_ASM_ANNOTATE") != nullptr;
    if (annotate) E.o << "  ; vcode " << cur_k << " " << phase << "\n";
  }
  bool spill_mask() {
    if (cur_k >= code.size()) return false;
    const Instr& in = code[cur_k];
    auto operand = [&](uint32_t id) {
      if (id == in.a || id == in.b || id == in.c) return true;
      if (in.op == K_LOOKUP) {
        if (id == in.p0) return true;
        for (uint32_t q = 0; q < 2 * in.c; q++)
          if (P.vaux[in.p1 + q] == id) return true;
      }
      return false;
    };
    int64_t best = -1;
    int32_t bl = -1;
    for (uint32_t id = 0; id < val.size(); id++) {
      const Val& x = val[id];
      if (!x.def || x.m.k != 2 || E.sref[x.m.s] != 1 || operand(id)) continue;
      const int32_t lu = id < last.size() ? last[id] : -1;
      if (lu > bl) {
        bl = lu;
        best = id;
      }
    }
    if (best < 0) return false;
    limb_of_bool((uint32_t)best);
    E.srelease(val[best].m);
    val[best].m = Mask{};
    return true;
  }
  // value `id` is dead: the cached differences it took part in go
  void eq_forget(uint32_t id) {
    for (auto it = eqdiff.begin(); it != eqdiff.end();) {
      if (it->first.first == id || it->first.second == id) {
        drop(it->second);
        it = eqdiff.erase(it);
      } else {
        ++it;
      }
    }
  }

  // MYTHGPU_JIT_ASM_NO_SIGNED_LIT=1: signed compares against literals through the borrow chain
  static bool no_signed_lit() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_SIGNED_LIT");
      return g && g[0] == '1';
    }();
    return on;
  }
  static bool no_mulshare() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_MULSHARE");
      return g && g[0] == '1';
    }();
    return on;
  }
  // a wave reads the hit word before its end-of-wave atomicMin (MYTHGPU_JIT_ASM_EXIT_SKIP=0: always
  // the atomic; profiles/r05s_rates_exit_skip.jsonl: C3's first tier 282 -> 435 G/s)
  static bool exit_skip() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_EXIT_SKIP");
      return !(g && g[0] == '0');
    }();
    return on;
  }
  static bool no_slt_clamp() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_SLT_CLAMP");
      return g && g[0] == '1';
    }();
    return on;
  }
  // the 32-bit clamp of x (La limbs, sign bit tb of the top limb): x_lo when the limbs above are
  // zero, else 0 for a negative x and ~0 for a positive one; held in hcache (owned by the caller: a
  // retained reference), or an unset limb when x's registers carry no allocation tags
  Limb clamp32(const std::vector<Limb>& rv, uint32_t La, uint32_t tb) {
    if (!(lvn_on && caches && !cond && !no_lvn())) return Limb{};
    std::vector<uint64_t> key{0xC1A3Full, tb};
    for (uint32_t j = 0; j < La; j++) {
      if (rv[j].reg() && (int)rv[j].v >= E.vfirst && !rv[j].g) return Limb{};
      key.push_back(lid(rv[j]));
    }
    auto it = hcache.find(key);
    if (it != hcache.end()) {
      h_last[key] = ++tick;
      E.retain(it->second);
      return it->second;
    }
    std::vector<std::pair<Limb, Limb>> hz;
    for (uint32_t j = 1; j < La; j++) hz.push_back({rv[j], Lit(0)});
    const Mask z = eq_mask(hz);
    const Limb t = fresh();
    if (tb == 31) E.valu("v_ashrrev_i32_e32 " + VL(t) + ", 31, " + VL(rv[La - 1]));
    else E.valu("v_bfe_i32 " + VL(t) + ", " + VL(rv[La - 1]) + ", " + std::to_string(tb) + ", 1");
    E.valu("v_not_b32_e32 " + VL(t) + ", " + VL(t));  // ~0 when x >= 0, else 0
    Limb lo = rv[0], tmp;
    if (lo.lit() && !inl(lo.v)) {
      tmp = vreg(lo);
      lo = tmp;
    }
    const Limb yv = fresh();
    if (z.k == 2) {
      E.valu("v_cndmask_b32_e64 " + VL(yv) + ", " + VL(t) + ", " + src(lo) + ", " + SP(z.s), {z.s, z.s + 1});
    } else {
      E.valu("v_mov_b32_e32 " + VL(yv) + ", " + (z.ones ? src(lo) : VL(t)));
    }
    E.srelease(z);
    drop(t);
    drop(tmp);
    E.retain(yv);
    hcache[key] = yv;
    h_last[key] = ++tick;
    for (uint32_t j = 0; j < La; j++)
      if (rv[j].reg() && (int)rv[j].v >= E.vfirst) hby.insert({rv[j].g, key});
    return yv;
  }
  // x <s y where one side is a literal K whose limbs above k are its sign extension (LASER's signed
  // bounds: 0 <s x, x <s 29, x <s -1): with neg = the register side's sign and hi = its limbs above k
  // equal K's, x <s K = neg | (hi & x_lo <u K_lo) for K >= 0, neg & (~hi | x_lo <u K_lo) for K < 0,
  // and K <s x the mirror image — a sign test, an equality over the high limbs and a compare of the
  // low ones, where the borrow chain runs through every limb with two wait states per link.  False
  // when no side qualifies (fewer than two register limbs above k)
  bool slt_literal(const std::vector<Limb>& x, const std::vector<Limb>& y, uint32_t w, Mask& out) {
    const uint32_t La = Lw(w), tb = (w - 1) & 31;
    const uint32_t topmask = tb == 31 ? 0xFFFFFFFFu : ((2u << tb) - 1u);
    for (int side = 0; side < 2; side++) {
      const std::vector<Limb>& kv = side ? x : y;  // the literal side
      const std::vector<Limb>& rv = side ? y : x;
      bool lit_all = true;
      for (uint32_t j = 0; j < La; j++) lit_all = lit_all && kv[j].lit();
      if (!lit_all) continue;
      const bool kneg = (kv[La - 1].v >> tb) & 1u;
      auto ext = [&](uint32_t j) { return kneg ? (j == La - 1 ? topmask : 0xFFFFFFFFu) : 0u; };
      int k = -1;  // highest limb of K that is not sign extension
      for (uint32_t j = 0; j < La; j++)
        if (kv[j].v != ext(j)) k = (int)j;
      if (k >= (int)La - 1) continue;
      std::vector<std::pair<Limb, Limb>> hi;
      uint32_t regs = 0;
      for (uint32_t j = (uint32_t)(k + 1); j < La; j++) {
        hi.push_back({rv[j], Lit(ext(j))});
        regs += rv[j].reg();
      }
      if (regs < 2 || !rv[La - 1].reg()) continue;
      // a value compared with many nonnegative literals below 2^32 - 1 (LASER's calldata reads: byte i
      // is ITE(i <s size, ..., 0) for every i): its 32-bit clamp y = (x < 2^32 ? x : x < 0 ? 0 : ~0)
      // once (cached), then K <s x = K <u y and x <s K = ~(K - 1 <u y), one compare each
      if (!kneg && k <= 0 && slt_many && !no_slt_clamp()) {
        const uint32_t K = kv[0].v;
        if (side == 1 ? K != 0xFFFFFFFFu : K != 0) {
          const Limb yc = clamp32(rv, La, tb);
          if (yc.reg()) {
            const Mask m = lt_mask({Lit(side == 1 ? K : K - 1)}, {yc}, 32, false);
            drop(yc);
            if (side == 1) {
              out = m;
            } else {
              out = mnot(m);
              E.srelease(m);
            }
            return true;
          }
        }
      }
      // the register side's sign: its top limb >= 2^tb
      Mask neg;
      if (tb == 31) {  // 0 >s top limb
        neg.k = 2;
        neg.s = E.salloc();
        E.valu("v_cmp_gt_i32_e64 " + SP(neg.s) + ", 0, " + VL(rv[La - 1]), {}, {neg.s, neg.s + 1});
      } else {
        neg = lt_mask({Lit((1u << tb) - 1u)}, {rv[La - 1]}, 32, false);
      }
      Mask eh;
      {
        const bool cacheable = lvn_on && caches && !cond && !no_lvn();
        std::vector<uint64_t> key;
        bool regs_ok = true;
        for (const auto& pr : hi) {
          key.push_back(lid(pr.first));
          key.push_back(lid(pr.second));
          if (pr.first.reg() && (int)pr.first.v >= E.vfirst && !pr.first.g) regs_ok = false;
        }
        auto it = cacheable && regs_ok ? hcache.find(key) : hcache.end();
        if (it != hcache.end()) {
          h_last[key] = ++tick;
          eh.k = 2;
          eh.s = E.salloc();
          E.valu("v_cmp_eq_u32_e64 " + SP(eh.s) + ", 0, " + VL(it->second), {}, {eh.s, eh.s + 1});
        } else {
          Limb keep{};
          eh = eq_mask(hi, cacheable && regs_ok ? &keep : nullptr);
          bool alias = false;  // an operand limb itself: a cached reference would pin its register
          for (const auto& pr : hi) alias = alias || (pr.first.reg() && pr.first.v == keep.v);
          if (keep.reg() && alias) {
            drop(keep);
          } else if (keep.reg()) {
            hcache[key] = keep;  // the reference eq_mask handed over
            h_last[key] = ++tick;
            for (const auto& pr : hi)
              if (pr.first.reg() && (int)pr.first.v >= E.vfirst) hby.insert({pr.first.g, key});
          }
        }
      }
      Mask lo;
      if (k < 0) {
        lo.k = 1;
        lo.ones = false;  // equal high limbs and no low ones: equal
      } else {
        lo = lt_mask(std::vector<Limb>(x.begin(), x.begin() + (k + 1)),
                     std::vector<Limb>(y.begin(), y.begin() + (k + 1)), 32u * (uint32_t)(k + 1), false);
      }
      Mask t, r;
      if (side == 0 && !kneg) {         // x < K, K >= 0: neg | (eh & lo)
        t = mop("and", eh, lo);
        r = mop("or", neg, t);
      } else if (side == 0) {           // x < K, K < 0: neg & ~(eh & ~lo)
        t = mop_andn(eh, lo);
        r = mop_andn(neg, t);
      } else if (!kneg) {               // K < x, K >= 0: ~(neg | (eh & ~lo))
        t = mop_andn(eh, lo);
        const Mask u = mop("or", neg, t);
        r = mnot(u);
        E.srelease(u);
      } else {                          // K < x, K < 0: ~(neg & ~(eh & lo))
        t = mop("and", eh, lo);
        const Mask u = mop_andn(neg, t);
        r = mnot(u);
        E.srelease(u);
      }
      E.srelease(t);
      E.srelease(neg);
      E.srelease(eh);
      E.srelease(lo);
      out = r;
      return true;
    }
    return false;
  }

  // x < y (unsigned) over La limbs, as a mask; sgn: the top limbs' bit (w-1)&31 flipped first
  Mask lt_mask(std::vector<Limb> x, std::vector<Limb> y, uint32_t w, bool sgn) {
    const uint32_t La = Lw(w);
    x.resize(La, Lit(0));
    y.resize(La, Lit(0));
    if (sgn && La > 1 && !no_signed_lit()) {
      Mask r;
      if (slt_literal(x, y, w, r)) return r;
    }
    std::vector<Limb> own;
    if (sgn) {
      const uint32_t f = 1u << ((w - 1) & 31);
      for (auto* v : {&x, &y}) {
        Limb& t = (*v)[La - 1];
        if (t.lit()) {
          t.v ^= f;
        } else {
          const Limb d = fresh();
          E.valu("v_xor_b32_e32 " + VL(d) + ", " + imm(f) + ", " + VL(t));
          t = d;
          own.push_back(d);
        }
      }
    }
    Mask m;
    // all-literal limbs from the top decide or drop out: find the lowest limb that matters
    if (La == 1) {
      const Limb a = x[0], b = y[0];
      if (a.lit() && b.lit()) {
        m.k = 1;
        m.ones = a.v < b.v;
      } else {
        m.k = 2;
        m.s = E.salloc();
        if (b.reg()) {
          if (a.lit() && !inl(a.v)) {
            E.valu("v_cmp_lt_u32_e32 vcc, " + src(a) + ", " + VL(b), {}, {kVCC, kVCC + 1});
            E.salu("s_mov_b64 " + SP(m.s) + ", vcc", {m.s, m.s + 1});
          } else {
            E.valu("v_cmp_lt_u32_e64 " + SP(m.s) + ", " + src(a) + ", " + VL(b), {}, {m.s, m.s + 1});
          }
        } else {
          if (!inl(b.v)) {
            E.valu("v_cmp_gt_u32_e32 vcc, " + src(b) + ", " + VL(a), {}, {kVCC, kVCC + 1});
            E.salu("s_mov_b64 " + SP(m.s) + ", vcc", {m.s, m.s + 1});
          } else {
            E.valu("v_cmp_gt_u32_e64 " + SP(m.s) + ", " + src(b) + ", " + VL(a), {}, {m.s, m.s + 1});
          }
        }
      }
      for (auto& d : own) drop(d);
      return m;
    }
    // a literal operand whose limbs above k are zero while the other's are registers (LASER's bounds
    // checks: x <= 20, 0 < x): the high limbs only need a zero test, x < K = (x_hi == 0) & (x_lo < K_lo)
    // and K < x = (x_hi != 0) | (K_lo < x_lo) — an OR-reduction instead of a borrow through every limb
    if (!sgn) {
      for (int side = 0; side < 2; side++) {
        const std::vector<Limb>& kv = side ? x : y;  // the literal side
        const std::vector<Limb>& rv = side ? y : x;
        int k = -1;  // highest nonzero limb of the literal side
        bool lit_all = true;
        for (uint32_t j = 0; j < La; j++) {
          if (!kv[j].lit()) lit_all = false;
          else if (kv[j].v) k = (int)j;
        }
        if (!lit_all) continue;
        std::vector<std::pair<Limb, Limb>> hz;
        for (uint32_t j = (uint32_t)(k + 1); j < La; j++)
          if (!(rv[j].lit() && rv[j].v == 0)) hz.push_back({rv[j], Lit(0)});
        uint32_t regs = 0;
        for (const auto& pr : hz) regs += pr.first.reg();
        if (regs < 2) continue;
        const uint32_t wl = 32u * (uint32_t)(k + 1);
        std::vector<Limb> xl(x.begin(), x.begin() + (k + 1)), yl(y.begin(), y.begin() + (k + 1));
        const Mask z = eq_mask(hz);  // the register side's high limbs are zero
        Mask lo;
        if (k < 0) {
          lo.k = 1;
          lo.ones = false;  // x_lo < y_lo over no limbs: 0 < 0
        } else {
          lo = lt_mask(xl, yl, wl, false);
        }
        Mask r;
        if (side == 0) {  // x < K
          r = mop("and", z, lo);
        } else {          // K < x
          const Mask nz = mnot(z);
          r = mop("or", nz, lo);
          E.srelease(nz);
        }
        E.srelease(z);
        E.srelease(lo);
        for (auto& d : own) drop(d);
        return r;
      }
    }
    // borrow chain of x - y; the difference itself is thrown away (v7)
    int borrow = 0;
    for (uint32_t j = 0; j < La; j++) {
      const Limb a = x[j], b = y[j];
      if (a.lit() && b.lit() && borrow >= 0) {
        borrow = ((uint64_t)a.v < (uint64_t)b.v + (uint64_t)borrow) ? 1 : 0;
        continue;
      }
      if (a.lit() && b.lit()) {
        // a borrow in VCC through literal limbs: equal ones pass it on, a larger minuend absorbs it,
        // a smaller one borrows regardless — no instruction
        if (a.v > b.v) borrow = 0;
        else if (a.v < b.v) borrow = 1;
        continue;
      }
      if (borrow == 1) {
        E.salu("s_mov_b64 vcc, -1", {kVCC, kVCC + 1});
        borrow = -1;
      }
      if (borrow == 0) {
        if (b.reg()) E.valu("v_sub_co_u32_e32 v7, vcc, " + src(a) + ", " + VL(b), {}, {kVCC, kVCC + 1});
        else E.valu("v_subrev_co_u32_e32 v7, vcc, " + src(b) + ", " + VL(a), {}, {kVCC, kVCC + 1});
      } else {
        Limb aa = a, bb = b, tmp, tmp2;
        if (!aa.reg() && !bb.reg()) {
          tmp = vreg(bb);
          bb = tmp;
        }
        if (aa.lit() && !inl(aa.v)) {  // VCC is on the constant bus
          tmp2 = vreg(aa);
          aa = tmp2;
        } else if (bb.lit() && !inl(bb.v)) {
          tmp2 = vreg(bb);
          bb = tmp2;
        }
        if (bb.reg())
          E.valu("v_subb_co_u32_e32 v7, vcc, " + src(aa) + ", " + VL(bb) + ", vcc", {kVCC, kVCC + 1}, {kVCC, kVCC + 1});
        else
          E.valu("v_subbrev_co_u32_e32 v7, vcc, " + src(bb) + ", " + VL(aa) + ", vcc", {kVCC, kVCC + 1},
                 {kVCC, kVCC + 1});
        drop(tmp);
        drop(tmp2);
      }
      borrow = -1;
    }
    for (auto& d : own) drop(d);
    if (borrow >= 0) {
      m.k = 1;
      m.ones = borrow == 1;
      return m;
    }
    m.k = 2;
    m.s = E.salloc();
    E.salu("s_mov_b64 " + SP(m.s) + ", vcc", {m.s, m.s + 1});
    return m;
  }

  Mask mnot(const Mask& a) {
    Mask m;
    if (a.k == 1) {
      m.k = 1;
      m.ones = !a.ones;
      return m;
    }
    m.k = 2;
    m.s = E.salloc();
    E.salu("s_not_b64 " + SP(m.s) + ", " + SP(a.s), {m.s, m.s + 1});
    return m;
  }
  // and / or / xor of masks
  Mask mop(const char* op, const Mask& a, const Mask& b) {
    Mask m;
    const std::string o = op;
    if (a.k == 1 && b.k == 1) {
      m.k = 1;
      m.ones = o == "and" ? (a.ones && b.ones) : o == "or" ? (a.ones || b.ones) : (a.ones != b.ones);
      return m;
    }
    if (a.k == 1 || b.k == 1) {
      const Mask& l = a.k == 1 ? a : b;
      const Mask& r = a.k == 1 ? b : a;
      if ((o == "and" && l.ones) || (o == "or" && !l.ones) || (o == "xor" && !l.ones)) {
        E.sretain(r);
        return r;
      }
      if (o == "and" || o == "or") {
        m.k = 1;
        m.ones = o == "or";
        return m;
      }
      return mnot(r);  // xor with all ones
    }
    m.k = 2;
    m.s = E.salloc();
    E.salu("s_" + o + "_b64 " + SP(m.s) + ", " + SP(a.s) + ", " + SP(b.s), {m.s, m.s + 1});
    return m;
  }

  // per-limb select through VCC (= the mask, already moved there): c ? t : f
  Limb sel(const Limb& t, const Limb& f) {
    if (t == f) {
      E.retain(t);
      return t;
    }
    if (t.k == LU || f.k == LU) fail("internal: a limb the demand analysis dropped was read");
    // VCC is on the constant bus already: a literal operand must come through a VGPR
    Limb tt = t, ff = f, tmp, tmp2;
    if (!tt.reg()) {
      tmp = vreg(tt);
      tt = tmp;
    }
    if (ff.lit() && !inl(ff.v)) {
      tmp2 = vreg(ff);
      ff = tmp2;
    }
    const Limb d = fresh();
    E.valu("v_cndmask_b32_e32 " + VL(d) + ", " + src(ff) + ", " + VL(tt) + ", vcc", {kVCC, kVCC + 1});
    drop(tmp);
    drop(tmp2);
    return d;
  }
  // m ? t : f with the mask in an SGPR pair (VOP3: the mask is the one constant-bus operand, so a
  // literal that is not an inline constant comes through a VGPR)
  static bool no_ite_e64() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_ITE_E64");
      return g && g[0] == '1';
    }();
    return on;
  }
  Limb sel_mask(const Limb& t, const Limb& f, const Mask& m) {
    if (t == f) {
      E.retain(t);
      return t;
    }
    if (t.k == LU || f.k == LU) fail("internal: a limb the demand analysis dropped was read");
    Limb tt = t, ff = f, tmp, tmp2;
    if (tt.lit() && !inl(tt.v)) {
      tmp = vreg(tt);
      tt = tmp;
    }
    if (ff.lit() && !inl(ff.v)) {
      tmp2 = vreg(ff);
      ff = tmp2;
    }
    const Limb d = fresh();
    E.valu("v_cndmask_b32_e64 " + VL(d) + ", " + src(ff) + ", " + src(tt) + ", " + SP(m.s), {m.s, m.s + 1});
    drop(tmp);
    drop(tmp2);
    return d;
  }
  void mask_to_vcc(const Mask& m) {
    if (m.k == 2) E.salu("s_mov_b64 vcc, " + SP(m.s), {kVCC, kVCC + 1});
    else E.salu(std::string("s_mov_b64 vcc, ") + (m.ones ? "-1" : "0"), {kVCC, kVCC + 1});
  }

  // ---------------------------------------------------------------------------------------
  // the candidate generator (GEN3, include/mythgpu.h; the same function as gen_value in
  // jit.cpp, engine.hip and oracle/bveval.c)
  // ---------------------------------------------------------------------------------------
  // per-lane hash grnd(c, j) into a fresh VGPR
  // (x ^ salt) ^ ((x ^ salt) >> 16) = (x ^ (x >> 16)) ^ (salt ^ (salt >> 16)): v4 holds the group-lane
  // key's x ^ (x >> 16), folded once per group (kernel()), so each draw XORs in its salt's fold — one
  // VALU per draw instead of two.  MYTHGPU_JIT_ASM_NO_KFOLD=1: the fold per draw
  static bool no_kfold() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_KFOLD");
      return g && g[0] == '1';
    }();
    return on;
  }
  Limb grnd(uint32_t c, uint32_t j, const Limb* into = nullptr) {
    const Limb d = into ? *into : fresh(), t = fresh();
    const uint32_t salt = gsalt(c, j);
    if (no_kfold()) {
      E.valu("v_xor_b32_e32 " + VL(d) + ", " + imm(salt) + ", v4");
      E.valu("v_xor_b32_sdwa " + VL(d) + ", " + VL(d) + ", " + VL(d) +
             " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1");
    } else {
      E.valu("v_xor_b32_e32 " + VL(d) + ", " + imm(salt ^ (salt >> 16)) + ", v4");
    }
    E.valu("v_mul_u32_u24_e32 " + VL(d) + ", 0x9e3779, " + VL(d));
    E.valu("v_lshrrev_b32_e32 " + VL(t) + ", 15, " + VL(d));
    E.valu("v_xad_u32 " + VL(d) + ", " + VL(t) + ", " + VL(d) + ", v5");
    drop(t);
    return d;
  }
  // the group's choice word of coordinate c -> SGPR s
  void gwsel(uint32_t c, int s) {
    E.salu("s_xor_b32 " + S(s) + ", s36, " + hexs(gsalt(c, 0xFFFEu)), {s});
    E.salu("s_mul_i32 " + S(s) + ", " + S(s) + ", 0x9e3779b1", {s});
    E.salu("s_add_u32 " + S(s) + ", " + S(s) + ", s37", {s});
  }
  // UNIFORM raw limbs masked to `bits`
  // tgt (MIXED branches): the coordinate's output registers, written directly (put then moves nothing)
  std::vector<Limb> uniform_limbs(uint32_t c, uint32_t Lc, uint32_t bits, const std::vector<Limb>* tgt = nullptr) {
    const uint32_t n = std::min(Lc, (bits + 31) / 32);
    if (tgt) {
      std::vector<Limb> r(*tgt);
      for (uint32_t j = 0; j < n; j++) {
        if (j < 2) {
          grnd(c, j, &r[j]);
        } else {
          const uint32_t s = (7u * j + 3u) % 31u + 1u;
          E.valu("v_alignbit_b32 " + VL(r[j]) + ", " + VL(r[j - 1]) + ", " + VL(r[j - 2]) + ", " + std::to_string(s));
          E.valu("v_add_u32_e32 " + VL(r[j]) + ", " + VL(r[j - 2]) + ", " + VL(r[j]));
        }
      }
      // the raw chain is complete: mask the top limb in place, zero the limbs above
      for (uint32_t j = 0; j < Lc; j++) {
        const uint32_t lo = 32 * j;
        const uint32_t m = lo >= bits ? 0u : (bits - lo >= 32 ? 0xFFFFFFFFu : ((1u << (bits - lo)) - 1u));
        if (j >= n || m == 0) E.valu("v_mov_b32_e32 " + VL(r[j]) + ", 0");
        else if (m != 0xFFFFFFFFu) E.valu("v_and_b32_e32 " + VL(r[j]) + ", " + imm(m) + ", " + VL(r[j]));
      }
      return r;
    }
    std::vector<Limb> u(n);
    for (uint32_t j = 0; j < n; j++) {
      if (j < 2) {
        u[j] = grnd(c, j);
      } else {
        const uint32_t s = (7u * j + 3u) % 31u + 1u;
        const Limb d = fresh();
        E.valu("v_alignbit_b32 " + VL(d) + ", " + VL(u[j - 1]) + ", " + VL(u[j - 2]) + ", " + std::to_string(s));
        E.valu("v_add_u32_e32 " + VL(d) + ", " + VL(u[j - 2]) + ", " + VL(d));
        u[j] = d;
      }
    }
    std::vector<Limb> r(Lc, Lit(0));
    for (uint32_t j = 0; j < Lc; j++) {
      const uint32_t lo = 32 * j;
      const uint32_t m = lo >= bits ? 0u : (bits - lo >= 32 ? 0xFFFFFFFFu : ((1u << (bits - lo)) - 1u));
      if (j >= n || m == 0) continue;
      r[j] = and_lit(u[j], m);
    }
    for (auto& x : u) drop(x);
    return r;
  }
  // lo + x for x < (maxadd << sh) + 1: the number of low limbs that can differ (jit.cpp reach_limbs)
  static uint32_t reach_limbs(const uint32_t* lo, uint32_t Lc, uint64_t maxadd, uint32_t sh) {
    std::vector<uint32_t> add(Lc + 3, 0u);
    const uint32_t q = sh / 32, r = sh % 32;
    const unsigned __int128 x = (unsigned __int128)maxadd << r;
    for (uint32_t t = 0; t < 3 && q + t < Lc + 3; t++) add[q + t] = (uint32_t)(x >> (32 * t));
    for (uint32_t j = Lc; j < Lc + 3; j++)
      if (add[j]) return Lc;
    uint64_t cy = 0;
    uint32_t k = 0;
    for (uint32_t j = 0; j < Lc; j++) {
      const uint64_t t = (uint64_t)lo[j] + add[j] + cy;
      if ((uint32_t)t != lo[j]) k = j + 1;
      cy = t >> 32;
    }
    return cy ? Lc : k;
  }
  // lo (literal limbs) + off (limbs, low limbs only), chain over the first k limbs
  std::vector<Limb> add_lit(const uint32_t* lo, uint32_t Lc, const std::vector<Limb>& off, uint32_t k) {
    std::vector<Limb> a(k), b(k);
    for (uint32_t j = 0; j < k; j++) {
      a[j] = Lit(lo[j]);
      b[j] = j < off.size() ? off[j] : Lit(0);
    }
    std::vector<Limb> r = add_chain(a, b, k, false);
    r.resize(Lc);
    for (uint32_t j = k; j < Lc; j++) r[j] = Lit(lo[j]);
    return r;
  }
  // high 32 bits of x * c (c a literal)
  Limb mulhi_lit(const Limb& x, uint32_t c) {
    if (x.lit()) return Lit((uint32_t)(((uint64_t)x.v * c) >> 32));
    const Limb d = fresh();
    if (inl(c)) {
      E.valu("v_mul_hi_u32 " + VL(d) + ", " + VL(x) + ", " + imm(c));
    } else {
      E.salu("s_mov_b32 s41, " + hexs(c), {41});
      E.valu("v_mul_hi_u32 " + VL(d) + ", " + VL(x) + ", s41", {41});
    }
    return d;
  }

  // dictionary entry `idx` (VGPR) of the n-entry table at G[off] (width w)
  // (upto: only limbs below it — the others come back as literal zeros, unread by the caller)
  std::vector<Limb> dict(uint32_t off, uint32_t n, uint32_t w, const Limb& idx, const std::vector<Limb>* tgt = nullptr,
                         uint32_t upto = 64) {
    const uint32_t Lc = Lw(w), Lu = std::min(Lc, upto);
    std::vector<Limb> r(Lc, Lit(0));
    auto dst = [&](uint32_t j) { return tgt ? (*tgt)[j] : fresh(); };
    if (w <= 32 && n && (uint64_t)n * w <= 32) {  // packed in one literal: one bit-field extract
      uint32_t pack = 0;
      const uint32_t m = w == 32 ? 0xFFFFFFFFu : ((1u << w) - 1u);
      for (uint32_t e2 = 0; e2 < n; e2++) pack |= (G[off + e2] & m) << (e2 * w);
      const Limb sh = fresh(), d = dst(0);
      E.valu("v_mul_u32_u24_e32 " + VL(sh) + ", " + imm(w) + ", " + VL(idx));
      E.salu("s_mov_b32 s41, " + hexs(pack), {41});
      E.valu("v_bfe_u32 " + VL(d) + ", s41, " + VL(sh) + ", " + std::to_string(w), {41});
      drop(sh);
      r[0] = d;
      return r;
    }
    if (n <= 4 && !lds_base.count(off)) {  // selects over the entries' literals
      std::vector<Mask> ms;
      for (uint32_t e2 = 0; e2 + 1 < n; e2++) {
        Mask m;
        m.k = 2;
        m.s = E.salloc();
        E.valu("v_cmp_ne_u32_e64 " + SP(m.s) + ", " + std::to_string(e2) + ", " + VL(idx), {}, {m.s, m.s + 1});
        ms.push_back(m);
      }
      // the select chain over entries e..n-1 of limb j, shared between limbs whose entries agree there
      // (the actor dictionary: two of three addresses repeat one word in every limb)
      std::map<std::vector<uint32_t>, Limb> memo;  // each entry holds one reference
      std::function<Limb(uint32_t, uint32_t)> chain = [&](uint32_t j, uint32_t e) -> Limb {
        std::vector<uint32_t> key{e};
        for (uint32_t k = e; k < n; k++) key.push_back(G[off + k * Lc + j]);
        auto it = memo.find(key);
        if (it != memo.end()) {
          E.retain(it->second);
          return it->second;
        }
        Limb cur;
        if (e + 1 == n) {
          cur = vreg(Lit(G[off + e * Lc + j]));
        } else {
          const Limb rest = chain(j, e + 1);
          const uint32_t lv = G[off + e * Lc + j];
          // lanes whose index is not e keep rest (src1), the others take the literal (src0)
          const Limb lvr = inl(lv) ? Lit(lv) : vreg(Lit(lv));  // VCC already uses the constant bus
          cur = fresh();
          E.valu("v_cndmask_b32_e64 " + VL(cur) + ", " + src(lvr) + ", " + VL(rest) + ", " + SP(ms[e].s),
                 {ms[e].s, ms[e].s + 1});
          drop(lvr);
          drop(rest);
        }
        memo[key] = cur;
        E.retain(cur);
        return cur;
      };
      for (uint32_t j = 0; j < Lu; j++) {
        bool same = true;
        for (uint32_t e2 = 1; e2 < n && same; e2++) same = G[off + e2 * Lc + j] == G[off + j];
        if (same) {
          r[j] = Lit(G[off + j]);
          continue;
        }
        const Limb rest = chain(j, 1);
        const uint32_t lv = G[off + j];
        const Limb lvr = inl(lv) ? Lit(lv) : vreg(Lit(lv));
        const Limb d = dst(j);
        E.valu("v_cndmask_b32_e64 " + VL(d) + ", " + src(lvr) + ", " + VL(rest) + ", " + SP(ms[0].s),
               {ms[0].s, ms[0].s + 1});
        drop(lvr);
        drop(rest);
        r[j] = d;
      }
      for (auto& kv : memo) drop(kv.second);
      for (auto& m : ms) E.srelease(m);
      return r;
    }
    auto lb = lds_base.find(off);
    if (lb != lds_base.end() && lds_pairs()) {  // pairs: limbs (2p, 2p+1) at word base + 2pn + 2 idx
      const Limb va = fresh();
      E.valu("v_lshlrev_b32_e32 " + VL(va) + ", 3, " + VL(idx));
      auto varies = [&](uint32_t j) {
        if (j >= Lu) return false;
        for (uint32_t e2 = 1; e2 < n; e2++)
          if (G[off + e2 * Lc + j] != G[off + j]) return true;
        return false;
      };
      bool any = false;
      for (uint32_t j = 0; j < Lu; j += 2) {
        const bool a0 = varies(j), a1 = j + 1 < Lc && varies(j + 1);
        if (!a0) r[j] = Lit(G[off + j]);
        if (j + 1 < Lc && !a1) r[j + 1] = Lit(G[off + j + 1]);
        if (!a0 && !a1) continue;
        const uint32_t byte = (lb->second + j * n) * 4;
        any = true;
        if (a0 && a1) {
          Limb d0, d1;
          if (tgt) {
            d0 = (*tgt)[j];
            d1 = (*tgt)[j + 1];
          } else {
            const uint32_t rr = E.valloc2();
            d0 = Limb{LR, rr, E.vgen[rr]};
            d1 = Limb{LR, rr + 1, E.vgen[rr + 1]};
          }
          if ((d0.v & 1u) == 0 && d1.v == d0.v + 1) {
            E.mem("ds_read_b64 " + VP(d0.v) + ", " + VL(va) + " offset:" + std::to_string(byte));
          } else {  // a target pair the allocator could not align
            E.mem("ds_read_b32 " + VL(d0) + ", " + VL(va) + " offset:" + std::to_string(byte));
            E.mem("ds_read_b32 " + VL(d1) + ", " + VL(va) + " offset:" + std::to_string(byte + 4));
          }
          r[j] = d0;
          r[j + 1] = d1;
          if (!no_lds_defer()) {
            E.lds_pending.insert((int)d0.v);
            E.lds_pending.insert((int)d1.v);
          }
        } else {
          const uint32_t q = a0 ? j : j + 1;
          const Limb d = dst(q);
          E.mem("ds_read_b32 " + VL(d) + ", " + VL(va) + " offset:" + std::to_string(byte + 4 * (q - j)));
          r[q] = d;
          if (!no_lds_defer()) E.lds_pending.insert((int)d.v);
        }
      }
      if (any && no_lds_defer()) E.ctl("s_waitcnt lgkmcnt(0)");
      drop(va);
      return r;
    }
    if (lb != lds_base.end()) {  // from the LDS copy: word base + j * n + idx
      const Limb va = fresh();
      E.valu("v_lshlrev_b32_e32 " + VL(va) + ", 2, " + VL(idx));
      bool any = false;
      for (uint32_t j = 0; j < Lu; j++) {
        bool same = true;
        for (uint32_t e2 = 1; e2 < n && same; e2++) same = G[off + e2 * Lc + j] == G[off + j];
        if (same) {
          r[j] = Lit(G[off + j]);
          continue;
        }
        const Limb d = dst(j);
        E.mem("ds_read_b32 " + VL(d) + ", " + VL(va) + " offset:" + std::to_string((lb->second + j * n) * 4));
        r[j] = d;
        any = true;
        if (!no_lds_defer()) E.lds_pending.insert((int)d.v);
      }
      if (any && no_lds_defer()) E.ctl("s_waitcnt lgkmcnt(0)");
      drop(va);  // (the address register may be reused at once: a load read its address at issue)
      return r;
    }
    // gathers from the generator constants (s[4:5]): byte offset (off + idx * Lc + j) * 4
    const Limb vo = fresh();
    E.valu("v_mul_u32_u24_e32 " + VL(vo) + ", " + imm(4 * Lc) + ", " + VL(idx));
    bool any = false;
    for (uint32_t j = 0; j < Lu; j++) {
      bool same = true;
      for (uint32_t e2 = 1; e2 < n && same; e2++) same = G[off + e2 * Lc + j] == G[off + j];
      if (same) {
        r[j] = Lit(G[off + j]);
        continue;
      }
      const uint32_t byte = (off + j) * 4;
      const Limb d = dst(j);
      if (byte < 4096) {
        E.mem("global_load_dword " + VL(d) + ", " + VL(vo) + ", s[4:5] offset:" + std::to_string(byte));
      } else {
        const Limb t = fresh();
        E.valu("v_add_u32_e32 " + VL(t) + ", " + hexs(byte) + ", " + VL(vo));
        E.mem("global_load_dword " + VL(d) + ", " + VL(t) + ", s[4:5]");
        drop(t);
      }
      r[j] = d;
      any = true;
    }
    if (any) E.ctl("s_waitcnt vmcnt(0)");
    drop(vo);
    return r;
  }

  // e = ((h >> 16) * n) >> 16
  // entry ((h >> 16) * n) >> 16: for n < 256 the high half of the 24-bit product (h >> 16) * (n << 16),
  // one v_mul_hi_u32_u24 for the multiply and the shift (MYTHGPU_JIT_ASM_NO_MULHI24=1: three VALU)
  static bool aligned_mad() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_ALIGNED_MAD");
      return !(g && g[0] == '0');
    }();
    return on;
  }
  static bool no_mulhi24() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_MULHI24");
      return g && g[0] == '1';
    }();
    return on;
  }
  Limb dict_index(const Limb& h, uint32_t n) {
    const Limb e2 = fresh();
    E.valu("v_lshrrev_b32_e32 " + VL(e2) + ", 16, " + VL(h));
    if (n < 256 && !no_mulhi24()) {
      E.valu("v_mul_hi_u32_u24_e32 " + VL(e2) + ", " + imm(n << 16) + ", " + VL(e2));
      return e2;
    }
    E.valu("v_mul_u32_u24_e32 " + VL(e2) + ", " + imm(n) + ", " + VL(e2));
    E.valu("v_lshrrev_b32_e32 " + VL(e2) + ", 16, " + VL(e2));
    return e2;
  }

  // write limbs r into the preassigned registers out (MIXED branches), releasing r
  void put(const std::vector<Limb>& out, std::vector<Limb>& r) {
    for (size_t j = 0; j < out.size(); j++) {
      const Limb x = j < r.size() ? r[j] : Lit(0);
      if (x == out[j]) continue;  // written in place (tgt): not a reference of its own
      E.valu("v_mov_b32_e32 " + VL(out[j]) + ", " + src(x));
      if (j < r.size()) drop(r[j]);
    }
    for (size_t j = out.size(); j < r.size(); j++) drop(r[j]);  // limbs above the ones generated
    r.clear();
  }

  // +/-(1 + (h & 1)) on the registers out, when (ws & 0xFFFF) < pdelta (scalar branch)
  void delta(const std::vector<Limb>& out, uint32_t c, uint32_t pdelta, int ws, const Limb* hknown) {
    CondScope cs_(*this);
    const std::string skip = E.newlab();
    E.salu("s_and_b32 s40, " + S(ws) + ", 0xffff", {40});
    E.salu("s_cmp_lt_u32 s40, " + imm(pdelta));
    E.ctl("s_cbranch_scc0 " + skip);
    Limb h = hknown ? *hknown : grnd(c, 0xFFFFu);
    if (hknown) E.retain(h);
    // mag = 1 + (h & 1); the sign sb = (h >> 1) & 1 as a mask; a0 = sb ? -mag : mag
    const Limb mag = fresh(), neg = fresh();
    Mask sb;
    sb.k = 2;
    sb.s = E.salloc();
    E.valu("v_and_b32_e32 " + VL(mag) + ", 1, " + VL(h));
    E.valu("v_add_u32_e32 " + VL(mag) + ", 1, " + VL(mag));
    E.valu("v_bfe_u32 " + VL(neg) + ", " + VL(h) + ", 1, 1");
    E.valu("v_cmp_ne_u32_e64 " + SP(sb.s) + ", 0, " + VL(neg), {}, {sb.s, sb.s + 1});
    E.valu("v_sub_u32_e32 " + VL(neg) + ", 0, " + VL(mag));
    E.valu("v_cndmask_b32_e64 " + VL(mag) + ", " + VL(mag) + ", " + VL(neg) + ", " + SP(sb.s), {sb.s, sb.s + 1});
    drop(neg);
    const uint32_t Lc = (uint32_t)out.size();
    E.valu("v_add_co_u32_e32 " + VL(out[0]) + ", vcc, " + VL(mag) + ", " + VL(out[0]), {}, {kVCC, kVCC + 1});
    drop(mag);
    if (Lc > 1) {
      // the high limbs change only in lanes whose low-limb carry differs from the step's sign
      const std::string done = E.newlab();
      E.salu("s_xor_b64 s[40:41], vcc, " + SP(sb.s), {40, 41});
      E.ctl("s_cbranch_scc0 " + done);
      const Limb ah = fresh();
      E.valu("v_cndmask_b32_e64 " + VL(ah) + ", 0, -1, " + SP(sb.s), {sb.s, sb.s + 1});
      for (uint32_t j = 1; j < Lc; j++)
        E.valu("v_addc_co_u32_e32 " + VL(out[j]) + ", vcc, " + VL(ah) + ", " + VL(out[j]) + ", vcc", {kVCC, kVCC + 1},
               {kVCC, kVCC + 1});
      drop(ah);
      E.label(done);
    }
    E.srelease(sb);
    drop(h);
    E.label(skip);
  }

  // mask to the width and the clamp record (MIXED: per branch, in place on out)
  // zero: limbs of out this branch knows to be zero (bit j = limb j)
  void finish(const std::vector<Limb>& out, uint32_t width, uint32_t clamp, uint64_t zero = 0) {
    const uint32_t Lc = (uint32_t)out.size();
    // a MIXED value generated to fewer limbs than the width (gen_value's want) has no top limb to mask
    // and no clamp (a clamp reads every limb: such values are generated whole)
    if (Lc < Lw(width)) return;
    if ((width & 31) && !(zero >> (Lc - 1) & 1))
      E.valu("v_and_b32_e32 " + VL(out[Lc - 1]) + ", " + imm(topmask(width)) + ", " + VL(out[Lc - 1]));
    if (!clamp) return;
    const uint32_t r = clamp - 1;
    const uint32_t span = G[r + Lc];
    bool lo_hi_zero = true;
    for (uint32_t j = 1; j < Lc; j++) lo_hi_zero = lo_hi_zero && G[r + j] == 0;
    if (lo_hi_zero && (span ? (uint64_t)G[r] + span <= (1ull << 32) : G[r] == 0)) {
      // lo < 2^32 and lo + span <= 2^32: in range iff the high limbs are zero and v0 - lo0 < span
      // (mod 2^32: a v0 below lo0 wraps to at least 2^32 - lo0 >= span) — no borrow chain
      std::vector<std::pair<Limb, Limb>> hz;
      for (uint32_t j = 1; j < Lc; j++)
        if (!(zero >> j & 1)) hz.push_back({out[j], Lit(0)});
      Mask bad;
      bad.k = 1;
      bad.ones = false;
      if (!hz.empty()) {
        const Mask z = eq_mask(hz);
        bad = mnot(z);
        E.srelease(z);
      }
      if (span) {
        Mask ge;
        ge.k = 2;
        ge.s = E.salloc();
        Limb d0 = out[0];
        if (G[r]) {
          d0 = fresh();
          E.valu("v_subrev_u32_e32 " + VL(d0) + ", " + imm(G[r]) + ", " + VL(out[0]));
        }
        if (inl(span)) {
          E.valu("v_cmp_le_u32_e64 " + SP(ge.s) + ", " + imm(span) + ", " + VL(d0), {}, {ge.s, ge.s + 1});
        } else {
          E.salu("s_mov_b32 s41, " + hexs(span), {41});
          E.valu("v_cmp_le_u32_e64 " + SP(ge.s) + ", s41, " + VL(d0), {41}, {ge.s, ge.s + 1});
        }
        if (G[r]) drop(d0);
        const Mask b2 = mop("or", bad, ge);
        E.srelease(ge);
        E.srelease(bad);
        bad = b2;
      }
      if (bad.k == 1 && !bad.ones) return;
      // clamped: lo0 + (span ? mulhi(v0, span) : v0) in limb 0 (no carry: below 2^32), zeros above
      Limb c0;
      if (span) {
        c0 = mulhi_lit(out[0], span);
        if (G[r]) E.valu("v_add_u32_e32 " + VL(c0) + ", " + imm(G[r]) + ", " + VL(c0));
      }
      mask_to_vcc(bad);
      if (span) {
        E.valu("v_cndmask_b32_e32 " + VL(out[0]) + ", " + VL(out[0]) + ", " + VL(c0) + ", vcc", {kVCC, kVCC + 1});
        drop(c0);
      }
      for (uint32_t j = 1; j < Lc; j++)
        if (!(zero >> j & 1))
          E.valu("v_cndmask_b32_e32 " + VL(out[j]) + ", " + VL(out[j]) + ", v6, vcc", {kVCC, kVCC + 1});
      E.srelease(bad);
      return;
    }
    const uint32_t k = reach_limbs(&G[r], Lc, span ? span - 1u : 0xFFFFFFFFull, 0);
    // in range: v - lo has no borrow, high limbs zero and low limb < span (span 0: 2^32)
    std::vector<Limb> v(out.begin(), out.end()), lo(Lc);
    for (uint32_t j = 0; j < Lc; j++) lo[j] = Lit(G[r + j]);
    // difference limbs (owned) and the borrow
    std::vector<Limb> dif = add_chain(v, lo, Lc, true);
    Mask bad;
    bad.k = 2;
    bad.s = E.salloc();
    E.salu("s_mov_b64 " + SP(bad.s) + ", vcc", {bad.s, bad.s + 1});  // borrow: v < lo
    std::vector<std::pair<Limb, Limb>> hz;
    for (uint32_t j = 1; j < Lc; j++) hz.push_back({dif[j], Lit(0)});
    if (!hz.empty()) {
      const Mask z = eq_mask(hz);  // high limbs of the difference zero
      const Mask nz = mnot(z);
      const Mask b2 = mop("or", bad, nz);
      E.srelease(z);
      E.srelease(nz);
      E.srelease(bad);
      bad = b2;
    }
    if (span) {
      Mask ge;
      ge.k = 2;
      ge.s = E.salloc();
      const Limb d0 = vreg(dif[0]);
      E.salu("s_mov_b32 s41, " + hexs(span), {41});
      E.valu("v_cmp_le_u32_e64 " + SP(ge.s) + ", s41, " + VL(d0), {41}, {ge.s, ge.s + 1});
      drop(d0);
      const Mask b2 = mop("or", bad, ge);
      E.srelease(ge);
      E.srelease(bad);
      bad = b2;
    }
    for (auto& d : dif) drop(d);
    // clamped value lo + (span ? mulhi(v0, span) : v0)
    std::vector<Limb> offv(1);
    offv[0] = span ? mulhi_lit(out[0], span) : out[0];
    if (!span) E.retain(out[0]);
    std::vector<Limb> cl = add_lit(&G[r], Lc, offv, k);
    drop(offv[0]);
    mask_to_vcc(bad);
    for (uint32_t j = 0; j < Lc; j++) {
      // out = bad ? clamped : out
      Limb t = cl[j], tmp;
      if (!t.reg()) {
        tmp = vreg(t);
        t = tmp;
      }
      E.valu("v_cndmask_b32_e32 " + VL(out[j]) + ", " + VL(out[j]) + ", " + VL(t) + ", vcc", {kVCC, kVCC + 1});
      drop(tmp);
      drop(cl[j]);
    }
    E.srelease(bad);
  }

  // fixed-bit record: v = (v & ~mask) | value
  void fixbits(std::vector<Limb>& r, uint32_t fix, bool in_place) {
    const uint32_t f = fix - 1, Lc = (uint32_t)r.size();
    for (uint32_t j = 0; j < Lc; j++) {
      const uint32_t m = G[f + j], v = G[f + Lc + j];
      if (!m) continue;
      if (in_place) {
        if (m == 0xFFFFFFFFu) {
          E.valu("v_mov_b32_e32 " + VL(r[j]) + ", " + imm(v));
          continue;
        }
        E.valu("v_and_b32_e32 " + VL(r[j]) + ", " + imm(~m) + ", " + VL(r[j]));
        if (v) E.valu("v_or_b32_e32 " + VL(r[j]) + ", " + imm(v) + ", " + VL(r[j]));
        continue;
      }
      if (m == 0xFFFFFFFFu || r[j].lit()) {
        const uint32_t x = r[j].lit() ? ((r[j].v & ~m) | v) : v;
        drop(r[j]);
        r[j] = Lit(x);
        continue;
      }
      const Limb a = and_lit(r[j], ~m);
      drop(r[j]);
      r[j] = a;
      if (v) {
        const Limb d = fresh();
        E.valu("v_or_b32_e32 " + VL(d) + ", " + imm(v) + ", " + VL(a));
        drop(a);
        r[j] = d;
      }
    }
  }

  // coordinate c's value (owned limbs).  want: the limbs the caller reads (bit j = limb j); a MIXED
  // value is generated only up to the highest of them that its fixed-bit record does not set whole
  // (the limbs above come back as literals: zeros, or the record's bits) — the same value in every
  // limb read, as each limb depends only on the limbs below it (carries, the UNIFORM chain) or on
  // none (dictionary entries).  A clamp reads every limb: such values are generated whole.
  // (C4: a COPY chain three MIXED levels deep whose every bit but one is fixed)
  std::vector<Limb> gen_value(uint32_t c, uint64_t want = ~0ull) {
    const GenSpec sp = specs.at(c);
    const uint32_t fix = sp.kind >> 8, kind = sp.kind & 0xFFu;
    const uint32_t width = P.coord_width.at(c), Lc = Lw(width);
    std::vector<Limb> r;
    switch (kind) {
      case MG_GEN_MIXED: {
        uint64_t wl = want & lowmask(Lc);
        if (fix)
          for (uint32_t j = 0; j < Lc; j++)
            if (G[fix - 1 + j] == 0xFFFFFFFFu) wl &= ~(1ull << j);
        const uint32_t Lg = (sp.p[6] || no_gen_want()) ? Lc : (wl ? 64u - (uint32_t)__builtin_clzll(wl) : 0u);
        if (Lg == 0) {  // nothing the caller reads is generated: the record's bits
          r.assign(Lc, Lit(0));
          if (fix) fixbits(r, fix, false);
          return r;
        }
        CondScope cs_(*this);
        std::vector<Limb> out(Lg);
        if (lds_pairs() && sp.p[1] && (sp.p[2] >> 16) && lds_base.count(sp.p[0])) {
          // the dictionary alternative reads limb pairs straight into these: even-aligned pairs
          for (uint32_t j = 0; j < Lg; j += 2) {
            if (j + 1 < Lg) {
              const uint32_t rr = E.valloc2();
              out[j] = Limb{LR, rr, E.vgen[rr]};
              out[j + 1] = Limb{LR, rr + 1, E.vgen[rr + 1]};
            } else {
              out[j] = fresh();
            }
          }
        } else {
          for (auto& x : out) x = fresh();
        }
        const uint32_t pc = sp.p[3] != MG_NONE ? (sp.p[2] & 0xFFFFu) : 0u;
        const uint32_t pd = sp.p[1] ? (sp.p[2] >> 16) : 0u;
        const uint32_t ps = sp.p[4] & 0xFFFFu;
        const uint32_t small_bits = std::min(width, sp.p[4] >> 16);
        const bool narrow = width <= MG_GEN_NARROW_BITS;
        const int ws = E.salloc();  // the choice word (one SGPR of a pair)
        gwsel(c, ws);
        const std::string end = E.newlab();
        auto uni = [&](uint32_t bitsn) {
          std::vector<Limb> u;
          if (narrow) {
            const Limb h = grnd(c, 0xFFFFu);
            u.assign(Lc, Lit(0));
            const uint32_t m = bitsn >= 32 ? 0xFFFFFFFFu : ((1u << bitsn) - 1u);
            u[0] = and_lit(h, m & 0xFFFFu);
            drop(h);
          } else {
            u = uniform_limbs(c, Lg, bitsn, &out);
          }
          put(out, u);
        };
        std::string next;
        bool any = false;
        auto branch = [&](uint32_t T) {  // take this alternative when ws < T << 16
          if (any) {
            E.ctl("s_branch " + end);
            E.label(next);
          }
          any = true;
          next = E.newlab();
          if (T < 65536u) {
            E.salu("s_cmp_lt_u32 " + S(ws) + ", " + hexs(T << 16));
            E.ctl("s_cbranch_scc0 " + next);
          }
        };
        note("mixed:key");
        if (pc) {
          branch(pc);
          note("mixed:copy");
          std::vector<Limb> s;
          // the source's value when it is still live and whole (a copy chain's inner source may
          // have been generated earlier and released after its last analysed use)
          auto it = cval.find(sp.p[3]);
          if (debug_live() && it != cval.end())
            fprintf(stderr, "asm copy source %u of %u: def %d need %llx\n", sp.p[3], c, (int)val[it->second].def,
                    (unsigned long long)need[it->second]);
          if (it != cval.end() && val[it->second].def &&
              (need[it->second] & lowmask(L(it->second))) == lowmask(L(it->second))) {
            s = val[it->second].l;
            for (auto& x : s) E.retain(x);
          } else {
            s = gen_value(sp.p[3], lowmask(Lg));
          }
          uint64_t zero = 0;  // limbs the copied value has as literal zeros (a delta may change them)
          for (uint32_t j = 0; j < Lc && !sp.p[5]; j++)
            if (j < s.size() && s[j].lit() && s[j].v == 0) zero |= 1ull << j;
          put(out, s);
          if (sp.p[5]) delta(out, c, sp.p[5], ws, nullptr);
          finish(out, width, sp.p[6], zero);
        }
        if (pd) {
          branch(pc + pd);
          note("mixed:dict");
          const Limb h = grnd(c, 0xFFFFu);
          const Limb ix = dict_index(h, sp.p[1]);
          std::vector<Limb> dv = dict(sp.p[0], sp.p[1], width, ix, &out, Lg);
          drop(ix);
          uint64_t zero = 0;  // limbs zero in every entry (a delta may change them)
          for (uint32_t j = 0; j < Lc && !sp.p[5]; j++)
            if (j < dv.size() && dv[j].lit() && dv[j].v == 0) zero |= 1ull << j;
          put(out, dv);
          if (sp.p[5]) delta(out, c, sp.p[5], ws, &h);
          drop(h);
          finish(out, width, sp.p[6], zero);
        }
        // limbs above `bitsn` are zero in the SMALL / UNIFORM values (narrow: everything above limb 0)
        auto zeros = [&](uint32_t bitsn) {
          uint64_t z = 0;
          for (uint32_t j = 0; j < Lc; j++)
            if ((narrow && j > 0) || 32 * j >= bitsn) z |= 1ull << j;
          return z;
        };
        if (ps) {
          branch(pc + pd + ps);
          note("mixed:small");
          uni(small_bits);
          finish(out, width, sp.p[6], zeros(small_bits));
        }
        if (any) {
          E.ctl("s_branch " + end);
          E.label(next);
        }
        note("mixed:uniform");
        uni(width);
        finish(out, width, sp.p[6], zeros(width));
        E.label(end);
        note("mixed:join");
        Mask wsm;
        wsm.k = 2;
        wsm.s = ws;
        E.srelease(wsm);
        // (every alternative masked its value to the width in finish)
        r.assign(Lc, Lit(0));
        for (uint32_t j = 0; j < Lg; j++) r[j] = out[j];
        if (fix) {
          // the record's bits: in place on the generated limbs; a generated limb the record sets
          // whole (below a wanted one) becomes its literal
          const uint32_t f = fix - 1;
          for (uint32_t j = 0; j < Lc; j++) {
            const uint32_t m = G[f + j], v = G[f + Lc + j];
            if (!m) continue;
            if (!r[j].reg() || m == 0xFFFFFFFFu) {
              drop(r[j]);
              r[j] = Lit(v);
              continue;
            }
            E.valu("v_and_b32_e32 " + VL(r[j]) + ", " + imm(~m) + ", " + VL(r[j]));
            if (v) E.valu("v_or_b32_e32 " + VL(r[j]) + ", " + imm(v) + ", " + VL(r[j]));
          }
        }
        return r;
      }
      case MG_GEN_DICT: {
        const Limb h = grnd(c, 0xFFFFu);
        const Limb ix = dict_index(h, sp.p[1]);
        drop(h);
        r = dict(sp.p[0], sp.p[1], width, ix);
        std::vector<Limb> rd = r;
        if (width & 31) mask_top(r, width);
        if (fix) fixbits(r, fix, false);
        // limbs still the entries' registers (not masked or fixed anew): dictionary limbs
        if (!no_dict_eq() && caches)
          for (uint32_t j = 0; j < r.size() && j < rd.size(); j++)
            if (r[j].reg() && r[j] == rd[j] && r[j].g == rd[j].g && !dlimb.count(r[j].g)) {
              DLimb dl;
              dl.off = sp.p[0];
              dl.n = sp.p[1];
              dl.Lc = Lc;
              dl.j = j;
              dl.idx = ix;
              E.retain(ix);
              dlimb[r[j].g] = dl;
            }
        drop(ix);
        return r;
      }
      case MG_GEN_RANGE: {
        const Limb rr = grnd(c, 0);
        std::vector<Limb> off(1);
        if (sp.p[1]) {
          off[0] = mulhi_lit(rr, sp.p[1]);
          drop(rr);
        } else {
          off[0] = rr;
        }
        const uint32_t k = reach_limbs(&G[sp.p[0]], Lc, sp.p[1] ? sp.p[1] - 1u : 0xFFFFFFFFull, 0);
        r = add_lit(&G[sp.p[0]], Lc, off, k);
        drop(off[0]);
        break;
      }
      case MG_GEN_ALIGNED: {
        const Limb rr = grnd(c, 0);
        Limb m;
        if (sp.p[2]) {
          m = mulhi_lit(rr, sp.p[2]);
          drop(rr);
        } else {
          m = rr;
        }
        const int32_t sh = (int32_t)sp.p[1];
        const uint32_t k = reach_limbs(&G[sp.p[0]], Lc, sp.p[2] ? sp.p[2] - 1u : 0xFFFFFFFFull, (uint32_t)sh);
        if (aligned_mad() && k == 2 && Lc >= 2 && sh > 0 && sh <= 6 && m.reg()) {
          // base + (m << sh) over two limbs as one m * 2^sh + base (v_mad_u64_u32, the base in s[40:41])
          // instead of two shifts and a carry pair (MYTHGPU_JIT_ASM_ALIGNED_MAD=0: those)
          const uint32_t rp = E.valloc2();
          E.salu("s_mov_b32 s40, " + hexs(G[sp.p[0]]), {40});
          E.salu("s_mov_b32 s41, " + hexs(G[sp.p[0] + 1]), {41});
          Mask cm;
          cm.k = 2;
          cm.s = E.salloc();
          E.valu("v_mad_u64_u32 v[" + std::to_string(rp) + ":" + std::to_string(rp + 1) + "], " + SP(cm.s) + ", " + VL(m) +
                     ", " + std::to_string(1 << sh) + ", s[40:41]",
                 {40, 41}, {cm.s, cm.s + 1});
          E.srelease(cm);
          drop(m);
          r.assign(Lc, Lit(0));
          r[0] = Limb{LR, rp, E.vgen[rp]};
          r[1] = Limb{LR, rp + 1, E.vgen[rp + 1]};
          for (uint32_t j = 2; j < Lc; j++) r[j] = Lit(G[sp.p[0] + j]);
          break;
        }
        std::vector<Limb> mw(Lc, Lit(0));
        for (uint32_t j = 0; j < Lc; j++) {
          const int32_t bit0 = (int32_t)(j * 32) - sh;
          if (bit0 <= -32 || bit0 >= 32) continue;
          const Limb d = fresh();
          if (bit0 < 0) E.valu("v_lshlrev_b32_e32 " + VL(d) + ", " + std::to_string(-bit0) + ", " + VL(m));
          else if (bit0 > 0) E.valu("v_lshrrev_b32_e32 " + VL(d) + ", " + std::to_string(bit0) + ", " + VL(m));
          else E.valu("v_mov_b32_e32 " + VL(d) + ", " + VL(m));
          mw[j] = d;
        }
        drop(m);
        r = add_lit(&G[sp.p[0]], Lc, mw, k);
        for (auto& x : mw) drop(x);
        break;
      }
      case MG_GEN_FIXED:
        r.resize(Lc);
        for (uint32_t j = 0; j < Lc; j++) r[j] = Lit(G[sp.p[0] + j]);
        break;
      default:  // UNIFORM / LAZY
        r = uniform_limbs(c, Lc, 32 * Lc);
        break;
    }
    if (width & 31) mask_top(r, width);
    if (fix) fixbits(r, fix, false);
    return r;
  }

  // ---------------------------------------------------------------------------------------
  // the program
  // ---------------------------------------------------------------------------------------
  void set(uint32_t d, std::vector<Limb> l) {
    Val& x = val[d];
    // limbs nobody reads are dropped (never computed where possible)
    for (size_t j = 0; j < l.size(); j++)
      if (!(need[d] >> j & 1) && l[j].k != LU) {
        drop(l[j]);
        l[j] = Limb{};
      }
    x.l = std::move(l);
    x.w = P.vwidth[d];
    x.def = true;
  }
  void set_mask(uint32_t d, const Mask& m) {
    Val& x = val[d];
    x.m = m;
    x.w = 1;
    x.def = true;
  }
  // ---- spills (eval kernels that do not fit 256 VGPRs otherwise) -----------------------------
  // A model read-back with many array reads at distinct symbolic keys (VMTests' calldata bytes: 32
  // canonicalising LOOKUPs, each comparing its key with every earlier one) keeps every key live to
  // the last lookup — 8 limbs each.  When the 256 VGPRs are taken and no cache entry is left, a live
  // value (width > 32, every register limb held by it alone, not read by the instruction being
  // emitted nor pinned by a key test in progress; the one whose last reader comes latest) goes to
  // LDS (ds_write per limb, the wave's slots at s35) and comes back on its next read (ds_read).
  // Spills happen outside branches only; a read of a spilled value under a branch fails the
  // kernel (the O3 kernel then).  Off unless the kernel fails without (jit_asm_source).
  // Slot layout, lane-major: lane l's slot k at s35 + 4 (S l + k), S = spill_stride() (odd, so the
  // 64 lanes of one access fall in distinct banks), one 16-bit ds offset of 4 k reaching every slot.
  // The slots of a workgroup's waves must fit the 160 KiB of LDS: at most 159 per wave with four
  // working waves; a read-back that needs more (VMTests' expXY: 63 live 256-bit keys) runs `solo` —
  // one working wave per 256-lane workgroup, the other three exit at once — with up to 639.
  bool spill_on = false;
  bool solo = false;
  uint32_t spill_stride() const { return spill_hwm | 1u; }
  uint32_t spill_cap() const { return ((160u * 1024u) / ((solo ? 1u : 4u) * 256u) - 1u) | 1u; }
  int vhard = 256;
  std::vector<std::vector<int>> spill_at;  // value id -> LDS slot of each register limb (-1 none); empty: resident
  std::vector<uint8_t> slot_busy;
  uint32_t spill_hwm = 0;
  Limb spill_v;                            // s35 + 4 * lane
  std::vector<uint32_t> pinned;            // the instruction's operands, and values pinned by PinScope
  struct PinScope {
    Gen& g;
    size_t n;
    PinScope(Gen& g_, std::initializer_list<uint32_t> ids) : g(g_), n(ids.size()) {
      for (uint32_t id : ids) g.pinned.push_back(id);
    }
    ~PinScope() { g.pinned.resize(g.pinned.size() - n); }
  };
  bool is_spilled(uint32_t id) const { return id < spill_at.size() && !spill_at[id].empty(); }
  bool spill_one() {
    if (!spill_on || cond) return false;
    int best = -1;
    int32_t bl = -1;
    for (uint32_t id = 0; id < val.size(); id++) {
      const Val& x = val[id];
      if (!x.def || is_spilled(id) || is_view(id) || P.vwidth[id] <= 32) continue;
      if (std::find(pinned.begin(), pinned.end(), id) != pinned.end()) continue;
      int regs = 0;
      bool own = true;
      for (const Limb& l : x.l)
        if (l.reg()) {
          regs++;
          own = own && (int)l.v >= E.vfirst && E.vref[l.v] == 1;
        }
      if (regs < 2 || !own) continue;
      const int32_t lu = id < last.size() ? last[id] : -1;
      if (lu > bl) {
        bl = lu;
        best = (int)id;
      }
    }
    if (best < 0) return false;
    Val& x = val[best];
    std::vector<int> at(x.l.size(), -1);
    for (size_t j = 0; j < x.l.size(); j++) {
      if (!x.l[j].reg()) continue;
      uint32_t sl = 0;
      while (sl < slot_busy.size() && slot_busy[sl]) sl++;
      if ((sl | 1u) > spill_cap()) fail("out of VGPRs (spill slots)");
      if (sl == slot_busy.size()) slot_busy.push_back(0);
      slot_busy[sl] = 1;
      spill_hwm = std::max(spill_hwm, sl + 1);
      E.mem("ds_write_b32 " + VL(spill_v) + ", " + VL(x.l[j]) + " offset:" + std::to_string(sl * 4u));
      at[j] = (int)sl;
    }
    E.ctl("s_waitcnt lgkmcnt(0)");  // the stores have read their registers
    for (size_t j = 0; j < x.l.size(); j++)
      if (at[j] >= 0) {
        drop(x.l[j]);
        x.l[j] = Limb{};
      }
    spill_at[best] = at;
    spills++;
    return true;
  }
  uint32_t spills = 0;
  void reload(uint32_t id) {
    if (cond) fail("a spilled value read under a branch");
    if (std::find(pinned.begin(), pinned.end(), id) == pinned.end())
      fail("internal: a spilled value read where it is not pinned");
    Val& x = val[id];
    const std::vector<int> at = spill_at[id];
    spill_at[id].clear();  // (pinned: not a victim of the allocations below)
    for (size_t j = 0; j < at.size(); j++) {
      if (at[j] < 0) continue;
      const Limb d = fresh();
      E.mem("ds_read_b32 " + VL(d) + ", " + VL(spill_v) + " offset:" + std::to_string((uint32_t)at[j] * 4u));
      x.l[j] = d;
    }
    E.ctl("s_waitcnt lgkmcnt(0)");
    for (int sl : at)
      if (sl >= 0) slot_busy[sl] = 0;
  }

  void kill(uint32_t id) {
    Val& x = val[id];
    if (is_spilled(id)) {
      for (int sl : spill_at[id])
        if (sl >= 0) slot_busy[sl] = 0;
      spill_at[id].clear();
    }
    for (auto& l : x.l) drop(l);
    x.l.clear();
    E.srelease(x.m);
    x.m = Mask{};
  }
  std::vector<Limb> limbs(uint32_t id, uint32_t n) {
    std::vector<Limb> r(n);
    for (uint32_t j = 0; j < n; j++) r[j] = limb(id, j);
    return r;
  }
  uint32_t demanded(uint32_t d) const { return need[d] ? 64 - (uint32_t)__builtin_clzll(need[d]) : 0; }

  // ---------------------------------------------------------------------------------------
  // data-dependent operators: variable shifts, division by a non-literal, EXP, Keccak-256.
  // Values are <= 256 bits here (the lowering's bound), so they live in <= 8 limbs; loops are
  // wave-uniform (trip counts are wave maxima found with ballots), per-lane work is predicated by
  // EXEC inside the loop (division) or by selects, and loop-carried values sit in registers
  // allocated before the loop and updated in place, so the allocator's state is the same at the
  // back edge as at the head.  Semantics: SMT-LIB total division (x / 0 = ~0, x % 0 = x), shifts
  // of w or more saturate, EVM EXP mod 2^w, Keccak-256 of the value's big-endian bytes.
  // ---------------------------------------------------------------------------------------
  // the divisor b is a literal below 2^32 (the limb-serial 2/1 path above)
  bool lit_divisor(uint32_t b, uint32_t Ld) const {
    const Instr* bd = def_of(b);
    bool ok = bd && bd->op == K_CONST;
    for (uint32_t j = 1; ok && j < Ld; j++) ok = P.consts[bd->p0 + j] == 0;
    return ok;
  }
  void drop_all(std::vector<Limb>& v) {
    for (auto& x : v) drop(x);
    v.clear();
  }
  // fresh registers holding x[0..n) (literal or missing limbs as their value / zero): loop state
  std::vector<Limb> own(const std::vector<Limb>& x, uint32_t n) {
    std::vector<Limb> r(n);
    for (uint32_t j = 0; j < n; j++) {
      const Limb s = j < x.size() && x[j].k != LU ? x[j] : Lit(0);
      r[j] = fresh();
      E.valu("v_mov_b32_e32 " + VL(r[j]) + ", " + src(s));
    }
    return r;
  }
  // a scalar SGPR (one of a pair) for loop counters and wave maxima
  int sreg() { return E.salloc(); }
  void sfree(int s) {
    Mask m;
    m.k = 2;
    m.s = s;
    E.srelease(m);
  }
  Mask mask_new() {
    Mask m;
    m.k = 2;
    m.s = E.salloc();
    return m;
  }
  // d = m ? t : f for VGPR operands (f/t may be the zero register)
  void vsel(const Limb& d, const Limb& f, const Limb& t, const Mask& m) {
    E.valu("v_cndmask_b32_e64 " + VL(d) + ", " + VL(f) + ", " + VL(t) + ", " + SP(m.s), {m.s, m.s + 1});
  }
  // a mask from one VALU compare of a VGPR with an inline constant or SGPR s41 (literal)
  Mask vcmp(const char* op, const Limb& a, uint32_t k) {
    Mask m = mask_new();
    if (inl(k)) {
      E.valu(std::string("v_cmp_") + op + "_u32_e64 " + SP(m.s) + ", " + VL(a) + ", " + imm(k), {}, {m.s, m.s + 1});
    } else {
      E.salu("s_mov_b32 s41, " + hexs(k), {41});
      E.valu(std::string("v_cmp_") + op + "_u32_e64 " + SP(m.s) + ", " + VL(a) + ", s41", {41}, {m.s, m.s + 1});
    }
    return m;
  }

  // bit length of a limb vector (0 for zero) into a fresh VGPR
  Limb bitlen(const std::vector<Limb>& x) {
    const Limb bl = fresh();
    E.valu("v_mov_b32_e32 " + VL(bl) + ", 0");
    for (uint32_t j = 0; j < x.size(); j++) {
      const Limb l = x[j];
      if (l.k == LU || (l.lit() && l.v == 0)) continue;
      if (l.lit()) {
        E.valu("v_mov_b32_e32 " + VL(bl) + ", " + imm(32 * j + 32 - (uint32_t)__builtin_clz(l.v)));
        continue;
      }
      const Limb t = fresh();
      E.valu("v_ffbh_u32_e32 " + VL(t) + ", " + VL(l));                      // leading zeros (~0 for 0)
      E.valu("v_sub_u32_e32 " + VL(t) + ", " + imm(32 * j + 32) + ", " + VL(t));
      const Mask nz = vcmp("ne", l, 0);
      vsel(bl, bl, t, nz);
      E.srelease(nz);
      drop(t);
    }
    return bl;
  }
  // the wave-uniform maximum of a per-lane value v < 2^bits into SGPR s (ballot binary search)
  void wave_max(const Limb& v, uint32_t bits, int s) {
    const int c = sreg();
    const Mask m = mask_new();
    E.salu("s_mov_b32 " + S(s) + ", 0", {s});
    for (int b = (int)bits - 1; b >= 0; b--) {
      E.salu("s_add_u32 " + S(c) + ", " + S(s) + ", " + imm(1u << b), {c});
      E.valu("v_cmp_ge_u32_e64 " + SP(m.s) + ", " + VL(v) + ", " + S(c), {c}, {m.s, m.s + 1});
      E.salu("s_cmp_lg_u64 " + SP(m.s) + ", 0");
      E.salu("s_cselect_b32 " + S(s) + ", " + S(c) + ", " + S(s), {s});
    }
    E.srelease(m);
    sfree(c);
  }

  // ---- shifts ------------------------------------------------------------------------------
  // x (owned registers, L limbs) shifted by whole limbs: q = s >> 5 per lane, barrel stages k =
  // 1, 2, 4, ... (a select per limb each); left: towards higher limbs, zero fill; right: fill f
  void limb_barrel(std::vector<Limb>& x, const Limb& s, bool left, const Limb& fill) {
    const uint32_t Lx = (uint32_t)x.size();
    const Limb q = fresh();
    E.valu("v_lshrrev_b32_e32 " + VL(q) + ", 5, " + VL(s));
    for (uint32_t k = 1; k <= Lx; k <<= 1) {
      const Limb t = fresh();
      E.valu("v_and_b32_e32 " + VL(t) + ", " + imm(k) + ", " + VL(q));
      const Mask on = vcmp("ne", t, 0);
      drop(t);
      if (left) {
        for (int i = (int)Lx - 1; i >= 0; i--) vsel(x[i], x[i], i >= (int)k ? x[i - k] : fill, on);
      } else {
        for (uint32_t i = 0; i < Lx; i++) vsel(x[i], x[i], i + k < Lx ? x[i + k] : fill, on);
      }
      E.srelease(on);
    }
    drop(q);
  }
  // x (owned) shifted within its limbs by s (a VGPR, 0 <= s <= 32 L): left or right with fill f
  // (a VGPR: the zero register or a sign word)
  void shift_limbs(std::vector<Limb>& x, const Limb& s, bool left, const Limb& fill) {
    const uint32_t Lx = (uint32_t)x.size();
    limb_barrel(x, s, left, fill);
    const Limb b = fresh();
    E.valu("v_and_b32_e32 " + VL(b) + ", 31, " + VL(s));
    if (left) {
      // x[i] = (x[i] << b) | (x[i-1] >> (32 - b)): alignbit by -b (mod 32), except b = 0
      const Limb nb = fresh(), t = fresh();
      E.valu("v_sub_u32_e32 " + VL(nb) + ", 0, " + VL(b));
      const Mask z = vcmp("eq", b, 0);
      for (int i = (int)Lx - 1; i >= 0; i--) {
        E.valu("v_alignbit_b32 " + VL(t) + ", " + VL(x[i]) + ", " + (i ? VL(x[i - 1]) : std::string("0")) + ", " + VL(nb));
        vsel(x[i], t, x[i], z);
      }
      E.srelease(z);
      drop(nb);
      drop(t);
    } else {
      for (uint32_t i = 0; i < Lx; i++)
        E.valu("v_alignbit_b32 " + VL(x[i]) + ", " + VL(i + 1 < Lx ? x[i + 1] : fill) + ", " + VL(x[i]) + ", " + VL(b));
    }
    drop(b);
  }
  // the shift amount of value b saturated to W, in a fresh VGPR
  Limb shift_amount(uint32_t bid, uint32_t W) {
    const uint32_t Lb = L(bid);
    const Limb b0 = limb(bid, 0), s = fresh();
    if (b0.lit()) E.valu("v_mov_b32_e32 " + VL(s) + ", " + imm(std::min(b0.v, W)));
    else E.valu("v_min_u32_e32 " + VL(s) + ", " + imm(W) + ", " + VL(b0));
    std::vector<std::pair<Limb, Limb>> hz;
    for (uint32_t j = 1; j < Lb; j++) hz.push_back({limb(bid, j), Lit(0)});
    if (!hz.empty()) {
      const Mask z = eq_mask(hz);  // every high limb zero
      if (z.k == 1) {
        if (!z.ones) E.valu("v_mov_b32_e32 " + VL(s) + ", " + imm(W));
      } else {
        const Limb wv = vreg(Lit(W));
        vsel(s, wv, s, z);
        drop(wv);
      }
      E.srelease(z);
    }
    return s;
  }
  // SHL / LSHR / ASHR of the width-W value a by value b
  std::vector<Limb> shift_var(uint32_t op, const std::vector<Limb>& a, uint32_t bid, uint32_t W) {
    const uint32_t La = Lw(W);
    std::vector<Limb> x = own(a, La);
    const Limb s = shift_amount(bid, W);
    Limb fill = Reg(6);
    if (op == K_ASHR) {
      // sign-extend the top limb, the fill word is its sign
      if (W & 31) E.valu("v_bfe_i32 " + VL(x[La - 1]) + ", " + VL(x[La - 1]) + ", 0, " + std::to_string(W & 31));
      fill = fresh();
      E.valu("v_ashrrev_i32_e32 " + VL(fill) + ", 31, " + VL(x[La - 1]));
    }
    shift_limbs(x, s, op == K_SHL, fill);
    if (op == K_ASHR) drop(fill);
    drop(s);
    mask_top(x, W);
    return x;
  }

  // ---- multiplication (low n limbs, schoolbook) ------------------------------------------------
  std::vector<Limb> mul_lo(const std::vector<Limb>& a, const std::vector<Limb>& b, uint32_t n) {
    std::vector<Limb> acc(n, Lit(0));  // owned
    for (uint32_t i = 0; i < n; i++) {
      const Limb x = i < a.size() ? a[i] : Lit(0);
      if (x.lit() && x.v == 0) continue;
      std::vector<Limb> lo(n, Lit(0)), hi(n, Lit(0));
      for (uint32_t j = 0; i + j < n; j++) {
        const Limb y = j < b.size() ? b[j] : Lit(0);
        if (y.lit() && y.v == 0) continue;
        if (x.lit() && y.lit()) {
          const uint64_t p = (uint64_t)x.v * y.v;
          lo[i + j] = Lit((uint32_t)p);
          if (i + j + 1 < n) hi[i + j + 1] = Lit((uint32_t)(p >> 32));
          continue;
        }
        const Limb vx = x.reg() ? x : y, ly = x.reg() ? y : x;
        const bool via_s41 = ly.lit() && !inl(ly.v);
        if (via_s41) E.salu("s_mov_b32 s41, " + hexs(ly.v), {41});
        const std::string so = via_s41 ? std::string("s41") : src(ly);
        Limb dl, dh;
        product(vx, so, via_s41, true, i + j + 1 < n, dl, dh);
        lo[i + j] = dl;
        if (i + j + 1 < n) hi[i + j + 1] = dh;
      }
      std::vector<Limb> s1 = add_chain(acc, lo, n, false);
      for (auto& t : acc) drop(t);
      for (auto& t : lo) drop(t);
      std::vector<Limb> s2 = add_chain(s1, hi, n, false);
      for (auto& t : s1) drop(t);
      for (auto& t : hi) drop(t);
      acc = s2;
    }
    return acc;
  }
  // low n limbs of a * a: the cross products a_i a_j (i < j) once, doubled by a one-bit shift, then
  // the squares a_i^2 added (bv_device.h sqr8): 16 products for 256 bits where mul_lo takes 36
  std::vector<Limb> sqr_lo(const std::vector<Limb>& a, uint32_t n) {
    auto at = [&](uint32_t i) { return i < a.size() ? a[i] : Lit(0); };
    std::vector<Limb> acc(n, Lit(0));  // owned
    for (uint32_t i = 0; 2 * i + 1 < n; i++) {
      const Limb x = at(i);
      if (x.lit() && x.v == 0) continue;
      std::vector<Limb> lo(n, Lit(0)), hi(n, Lit(0));
      for (uint32_t j = i + 1; i + j < n; j++) {
        const Limb y = at(j);
        if (y.lit() && y.v == 0) continue;
        if (x.lit() && y.lit()) {
          const uint64_t p = (uint64_t)x.v * y.v;
          lo[i + j] = Lit((uint32_t)p);
          if (i + j + 1 < n) hi[i + j + 1] = Lit((uint32_t)(p >> 32));
          continue;
        }
        const Limb vx = x.reg() ? x : y, ly = x.reg() ? y : x;
        const bool via_s41 = ly.lit() && !inl(ly.v);
        if (via_s41) E.salu("s_mov_b32 s41, " + hexs(ly.v), {41});
        const std::string so = via_s41 ? std::string("s41") : src(ly);
        Limb dl, dh;
        product(vx, so, via_s41, true, i + j + 1 < n, dl, dh);
        lo[i + j] = dl;
        if (i + j + 1 < n) hi[i + j + 1] = dh;
      }
      std::vector<Limb> s1 = add_chain(acc, lo, n, false);
      drop_all(acc);
      drop_all(lo);
      acc = add_chain(s1, hi, n, false);
      drop_all(s1);
      drop_all(hi);
    }
    // acc <<= 1 (limb n-1's top bit drops out)
    std::vector<Limb> dbl(n, Lit(0));
    for (int j = (int)n - 1; j >= 0; j--) {
      const Limb hi = acc[j], lo = j ? acc[j - 1] : Lit(0);
      if (hi.lit() && lo.lit()) {
        dbl[j] = Lit((hi.v << 1) | (lo.v >> 31));
        continue;
      }
      const Limb d = fresh();
      if (lo.lit() && lo.v == 0) E.valu("v_lshlrev_b32_e32 " + VL(d) + ", 1, " + VL(hi.reg() ? hi : vreg(hi)));
      else {
        const Limb h = v3(hi), l = v3(lo);
        E.valu("v_alignbit_b32 " + VL(d) + ", " + src(h) + ", " + src(l) + ", 31");
        drop(h);
        drop(l);
      }
      dbl[j] = d;
    }
    drop_all(acc);
    // the squares at limbs 2i, 2i + 1
    std::vector<Limb> sq(n, Lit(0));
    for (uint32_t i = 0; 2 * i < n; i++) {
      const Limb x = at(i);
      if (x.lit()) {
        const uint64_t p = (uint64_t)x.v * x.v;
        sq[2 * i] = Lit((uint32_t)p);
        if (2 * i + 1 < n) sq[2 * i + 1] = Lit((uint32_t)(p >> 32));
        continue;
      }
      Limb dl, dh;
      product(x, VL(x), false, true, 2 * i + 1 < n, dl, dh);
      sq[2 * i] = dl;
      if (2 * i + 1 < n) sq[2 * i + 1] = dh;
    }
    std::vector<Limb> r = add_chain(dbl, sq, n, false);
    drop_all(dbl);
    drop_all(sq);
    return r;
  }
  // dst[j] = v[j] (moves into loop-state registers; v released)
  void assign(const std::vector<Limb>& dst, std::vector<Limb>& v) {
    for (size_t j = 0; j < dst.size(); j++) {
      const Limb x = j < v.size() && v[j].k != LU ? v[j] : Lit(0);
      if (x == dst[j]) continue;
      E.valu("v_mov_b32_e32 " + VL(dst[j]) + ", " + src(x));
    }
    drop_all(v);
  }

  // ---- division ------------------------------------------------------------------------------
  // q, r of a / b (unsigned, width W) with SMT-LIB's total division: per lane, a restoring
  // division over the quotient's bits only (la - lb + 1 of them, la / lb the bit lengths, as
  // bv_device.h udivrem8), the remainder kept in NB limbs — NB the wave's widest divisor, one of
  // 1 / 2 / 4 / L, a uniform branch — and the loop run for the wave's longest quotient with
  // EXEC holding the lanes that still have steps
  void udivrem(const std::vector<Limb>& a_in, const std::vector<Limb>& b_in, uint32_t W, std::vector<Limb>& q,
               std::vector<Limb>& r) {
    CondScope cs_(*this);
    const uint32_t La = Lw(W), C = 32 * La;
    std::vector<Limb> a = a_in, b = b_in;
    a.resize(La, Lit(0));
    b.resize(La, Lit(0));
    note("udivrem:bitlen");
    const Limb la = bitlen(a), lb = bitlen(b);
    // n = la >= lb ? la - lb + 1 : 0
    const Limb n = fresh();
    E.valu("v_sub_u32_e32 " + VL(n) + ", " + VL(la) + ", " + VL(lb));
    E.valu("v_add_u32_e32 " + VL(n) + ", 1, " + VL(n));
    {
      Mask lt = mask_new();
      E.valu("v_cmp_lt_u32_e64 " + SP(lt.s) + ", " + VL(la) + ", " + VL(lb), {}, {lt.s, lt.s + 1});
      vsel(n, n, Reg(6), lt);
      E.srelease(lt);
      // b == 0: no steps either (the SMT-LIB result is substituted at the end) — a zero divisor would
      // otherwise run the wave for la + 1 steps (up to 257)
      const Mask z = vcmp("eq", lb, 0);
      vsel(n, n, Reg(6), z);
      E.srelease(z);
    }
    drop(la);
    note("udivrem:shift");
    // rem = a >> n, quo = a << (C - n)
    std::vector<Limb> rem = own(a, La), quo = own(a, La);
    shift_limbs(rem, n, false, Reg(6));
    {
      const Limb cn = fresh();
      E.valu("v_sub_u32_e32 " + VL(cn) + ", " + imm(C) + ", " + VL(n));
      shift_limbs(quo, cn, true, Reg(6));
      drop(cn);
    }
    // the divisor's limbs as registers for the subtraction
    std::vector<Limb> bv(La);
    for (uint32_t j = 0; j < La; j++) bv[j] = vreg(b[j]);
    note("udivrem:onelimb");
    // lanes whose divisor is one non-zero limb (x / 10**k, x / n for a small n): limb-serial long
    // division instead (div_one_limb), and out of the bit-serial loop below (n = 0)
    {
      std::vector<std::pair<Limb, Limb>> hz;
      for (uint32_t j = 1; j < La; j++) hz.push_back({b[j], Lit(0)});
      const Mask hiz = hz.empty() ? Mask{1, true, -1} : eq_mask(hz);
      Mask nz0;
      if (b[0].lit()) {
        nz0.k = 1;
        nz0.ones = b[0].v != 0;
      } else {
        nz0 = vcmp("ne", bv[0], 0);
      }
      const Mask one = mop("and", hiz, nz0);
      E.srelease(hiz);
      E.srelease(nz0);
      if (!(one.k == 1 && !one.ones)) {
        div_one_limb(a, bv[0], quo, rem, one);
        if (one.k == 1) E.valu("v_mov_b32_e32 " + VL(n) + ", 0");
        else vsel(n, n, Reg(6), one);
      }
      E.srelease(one);
    }
    note("udivrem:loop");
    const int sN = sreg(), sIt = sreg();
    wave_max(n, 9, sN);
    // NB: the wave's widest divisor in limbs (ballots over the divisor's limbs)
    const int sNB = sreg();
    E.salu("s_mov_b32 " + S(sNB) + ", 1", {sNB});
    {
      const Mask m = mask_new();
      for (uint32_t j = 1; j < La; j++) {
        if (b[j].lit() && b[j].v == 0) continue;
        if (b[j].lit()) {
          E.salu("s_mov_b32 " + S(sNB) + ", " + imm(j + 1), {sNB});
          continue;
        }
        E.valu("v_cmp_ne_u32_e64 " + SP(m.s) + ", 0, " + VL(bv[j]), {}, {m.s, m.s + 1});
        E.salu("s_cmp_lg_u64 " + SP(m.s) + ", 0");
        E.salu("s_cselect_b32 " + S(sNB) + ", " + imm(j + 1) + ", " + S(sNB), {sNB});
      }
      E.srelease(m);
    }
    std::vector<uint32_t> widths;
    for (uint32_t nb : {1u, 2u, 4u, La})
      if (nb <= La && std::find(widths.begin(), widths.end(), nb) == widths.end()) widths.push_back(nb);
    const std::string done = E.newlab();
    const Mask act = mask_new(), cm = mask_new(), ge = mask_new();
    for (size_t vi = 0; vi < widths.size(); vi++) {
      const uint32_t NB = widths[vi];
      const std::string next = E.newlab(), loop = E.newlab(), end = E.newlab();
      if (vi + 1 < widths.size()) {  // this variant serves the waves whose widest divisor has <= NB limbs
        E.salu("s_cmp_gt_u32 " + S(sNB) + ", " + imm(NB));
        E.ctl("s_cbranch_scc1 " + next);
      }
      E.salu("s_mov_b32 " + S(sIt) + ", 0", {sIt});
      E.label(loop);
      E.salu("s_cmp_ge_u32 " + S(sIt) + ", " + S(sN));
      E.ctl("s_cbranch_scc1 " + end);
      // lanes with a step left
      E.salu("s_mov_b64 exec, -1");
      E.valu("v_cmp_gt_u32_e64 " + SP(act.s) + ", " + VL(n) + ", " + S(sIt), {sIt}, {act.s, act.s + 1});
      E.salu("s_mov_b64 exec, " + SP(act.s));
      // (rem : quo) <<= 1: quo's top bit carries into rem, rem's top bit out (cm)
      for (uint32_t i = 0; i < La; i++) {
        if (i == 0) E.valu("v_add_co_u32_e32 " + VL(quo[0]) + ", vcc, " + VL(quo[0]) + ", " + VL(quo[0]), {}, {kVCC, kVCC + 1});
        else E.valu("v_addc_co_u32_e32 " + VL(quo[i]) + ", vcc, " + VL(quo[i]) + ", " + VL(quo[i]) + ", vcc", {kVCC, kVCC + 1}, {kVCC, kVCC + 1});
      }
      for (uint32_t i = 0; i < NB; i++)
        E.valu("v_addc_co_u32_e32 " + VL(rem[i]) + ", vcc, " + VL(rem[i]) + ", " + VL(rem[i]) + ", vcc", {kVCC, kVCC + 1}, {kVCC, kVCC + 1});
      E.salu("s_mov_b64 " + SP(cm.s) + ", vcc", {cm.s, cm.s + 1});
      // d = rem - b (NB limbs); ge = carry-out | no borrow
      std::vector<Limb> dd(NB);
      for (uint32_t i = 0; i < NB; i++) {
        dd[i] = fresh();
        if (i == 0) E.valu("v_sub_co_u32_e32 " + VL(dd[0]) + ", vcc, " + VL(rem[0]) + ", " + VL(bv[0]), {}, {kVCC, kVCC + 1});
        else E.valu("v_subb_co_u32_e32 " + VL(dd[i]) + ", vcc, " + VL(rem[i]) + ", " + VL(bv[i]) + ", vcc", {kVCC, kVCC + 1}, {kVCC, kVCC + 1});
      }
      E.salu("s_orn2_b64 " + SP(ge.s) + ", " + SP(cm.s) + ", vcc", {ge.s, ge.s + 1});
      for (uint32_t i = 0; i < NB; i++) vsel(rem[i], rem[i], dd[i], ge);
      drop_all(dd);
      // the quotient bit
      E.salu("s_mov_b64 vcc, " + SP(ge.s), {kVCC, kVCC + 1});
      E.valu("v_addc_co_u32_e32 " + VL(quo[0]) + ", vcc, 0, " + VL(quo[0]) + ", vcc", {kVCC, kVCC + 1}, {kVCC, kVCC + 1});
      E.salu("s_add_u32 " + S(sIt) + ", " + S(sIt) + ", 1", {sIt});
      E.ctl("s_branch " + loop);
      E.label(end);
      E.salu("s_mov_b64 exec, -1");
      if (vi + 1 < widths.size()) {
        E.ctl("s_branch " + done);
        E.label(next);
      }
    }
    E.label(done);
    E.salu("s_mov_b64 exec, -1");
    E.srelease(act);
    E.srelease(cm);
    E.srelease(ge);
    sfree(sN);
    sfree(sIt);
    sfree(sNB);
    drop(n);
    for (auto& x : bv) drop(x);
    note("udivrem:zero");
    // b == 0 (lb == 0): q = ~0 (to the width), r = a
    {
      const Mask z = vcmp("eq", lb, 0);
      for (uint32_t i = 0; i < La; i++) {
        const uint32_t ones = i == La - 1 ? topmask(W) : 0xFFFFFFFFu;
        const Limb o = vreg(Lit(ones));
        vsel(quo[i], quo[i], o, z);
        drop(o);
        const Limb ai = vreg(a[i]);
        vsel(rem[i], rem[i], ai, z);
        drop(ai);
      }
      E.srelease(z);
    }
    drop(lb);
    q = quo;
    r = rem;
  }
  // quo / rem of the lanes in mask `one` (divisor d = one non-zero limb): normalised long division,
  // one Moller-Granlund 2/1 step per limb (Moller & Granlund, "Improved division by invariant
  // integers", IEEE TC 2011, Alg. 4; as bv_device.h udivrem8's one-limb path), with the per-lane
  // reciprocal v = floor((2^64 - 1) / dn) - 2^32 of the normalised divisor dn computed exactly by 32
  // restoring steps (the numerator (~dn : 2^32 - 1) over dn: the quotient has 32 bits).  EXEC holds
  // the lanes of `one` throughout; quo / rem are written for them only
  void div_one_limb(const std::vector<Limb>& a, const Limb& d0, std::vector<Limb>& quo, std::vector<Limb>& rem,
                    const Mask& one) {
    const uint32_t La = (uint32_t)quo.size();
    const std::string skip = E.newlab();
    if (one.k == 2) {
      E.salu("s_mov_b64 exec, " + SP(one.s));
      E.ctl("s_cbranch_execz " + skip);
    }
    const Limb sh = fresh(), dn = fresh(), rv = fresh(), rr = fresh(), t = fresh(), q0 = fresh(), q1 = fresh();
    E.valu("v_ffbh_u32_e32 " + VL(sh) + ", " + VL(d0));
    E.valu("v_lshlrev_b32_e32 " + VL(dn) + ", " + VL(sh) + ", " + VL(d0));
    // rv = floor(((~dn) * 2^32 + 2^32 - 1) / dn): 32 steps of rem = 2 rem + 1, a carry-out or rem >= dn
    // subtracts dn and sets the quotient bit
    {
      const Mask c = mask_new(), g = mask_new();
      const int sK = sreg();
      E.valu("v_not_b32_e32 " + VL(rr) + ", " + VL(dn));
      E.valu("v_mov_b32_e32 " + VL(rv) + ", 0");
      E.salu("s_mov_b32 " + S(sK) + ", 32", {sK});
      const std::string loop = E.newlab();
      E.label(loop);
      E.valu("v_cmp_gt_i32_e64 " + SP(c.s) + ", 0, " + VL(rr), {}, {c.s, c.s + 1});  // top bit set
      E.valu("v_lshl_or_b32 " + VL(rr) + ", " + VL(rr) + ", 1, 1");
      E.valu("v_cmp_ge_u32_e64 " + SP(g.s) + ", " + VL(rr) + ", " + VL(dn), {}, {g.s, g.s + 1});
      E.salu("s_or_b64 " + SP(g.s) + ", " + SP(g.s) + ", " + SP(c.s), {g.s, g.s + 1});
      E.valu("v_sub_u32_e32 " + VL(t) + ", " + VL(rr) + ", " + VL(dn));
      vsel(rr, rr, t, g);
      E.salu("s_mov_b64 vcc, " + SP(g.s), {kVCC, kVCC + 1});
      E.valu("v_addc_co_u32_e32 " + VL(rv) + ", vcc, " + VL(rv) + ", " + VL(rv) + ", vcc", {kVCC, kVCC + 1},
             {kVCC, kVCC + 1});
      E.salu("s_add_u32 " + S(sK) + ", " + S(sK) + ", -1", {sK});
      E.salu("s_cmp_lg_u32 " + S(sK) + ", 0");
      E.ctl("s_cbranch_scc1 " + loop);
      E.srelease(c);
      E.srelease(g);
      sfree(sK);
    }
    // the dividend shifted left by sh into La + 1 limbs: xs[j] = ({a[j], a[j-1]} << sh) >> 32
    const Limb nsh = fresh();
    E.valu("v_sub_u32_e32 " + VL(nsh) + ", 0, " + VL(sh));
    const Mask z = vcmp("eq", sh, 0);
    std::vector<Limb> xs(La + 1);
    for (uint32_t j = 0; j <= La; j++) {
      const Limb hi = j < La ? vreg(a[j]) : Reg(6), lo = j ? vreg(a[j - 1]) : Reg(6);
      xs[j] = fresh();
      E.valu("v_alignbit_b32 " + VL(xs[j]) + ", " + VL(hi) + ", " + VL(lo) + ", " + VL(nsh));
      vsel(xs[j], xs[j], hi, z);
      drop(hi);
      drop(lo);
    }
    E.srelease(z);
    drop(nsh);
    const Mask M = mask_new();
    // the top word of the shifted dividend is below 2^sh <= dn: the first step's high word
    E.valu("v_mov_b32_e32 " + VL(rr) + ", " + VL(xs[La]));
    for (int32_t j = (int32_t)La - 1; j >= 0; j--) {
      const Limb& u0 = xs[j];
      // (q1:q0) = rv * rr + (rr + 1 : u0)
      E.valu("v_mul_lo_u32 " + VL(q0) + ", " + VL(rr) + ", " + VL(rv));
      E.valu("v_mul_hi_u32 " + VL(q1) + ", " + VL(rr) + ", " + VL(rv));
      E.valu("v_add_co_u32_e32 " + VL(q0) + ", vcc, " + VL(q0) + ", " + VL(u0), {}, {kVCC, kVCC + 1});
      E.valu("v_addc_co_u32_e32 " + VL(q1) + ", vcc, " + VL(q1) + ", " + VL(rr) + ", vcc", {kVCC, kVCC + 1},
             {kVCC, kVCC + 1});
      E.valu("v_add_u32_e32 " + VL(q1) + ", 1, " + VL(q1));
      // r = u0 - q1 dn (mod 2^32); r > q0: q1 - 1, r + dn; then r >= dn: q1 + 1, r - dn
      E.valu("v_mul_lo_u32 " + VL(t) + ", " + VL(q1) + ", " + VL(dn));
      E.valu("v_sub_u32_e32 " + VL(rr) + ", " + VL(u0) + ", " + VL(t));
      E.valu("v_cmp_gt_u32_e64 " + SP(M.s) + ", " + VL(rr) + ", " + VL(q0), {}, {M.s, M.s + 1});
      E.valu("v_add_u32_e32 " + VL(t) + ", -1, " + VL(q1));
      E.valu("v_add_u32_e32 " + VL(q0) + ", " + VL(dn) + ", " + VL(rr));
      vsel(q1, q1, t, M);
      vsel(rr, rr, q0, M);
      E.valu("v_cmp_le_u32_e64 " + SP(M.s) + ", " + VL(dn) + ", " + VL(rr), {}, {M.s, M.s + 1});
      E.valu("v_add_u32_e32 " + VL(t) + ", 1, " + VL(q1));
      E.valu("v_sub_u32_e32 " + VL(q0) + ", " + VL(rr) + ", " + VL(dn));
      vsel(q1, q1, t, M);
      vsel(rr, rr, q0, M);
      E.valu("v_mov_b32_e32 " + VL(quo[j]) + ", " + VL(q1));
    }
    E.srelease(M);
    E.valu("v_lshrrev_b32_e32 " + VL(rem[0]) + ", " + VL(sh) + ", " + VL(rr));
    for (uint32_t j = 1; j < La; j++) E.valu("v_mov_b32_e32 " + VL(rem[j]) + ", 0");
    for (auto& x : xs) drop(x);
    for (const Limb& x : {sh, dn, rv, rr, t, q0, q1}) drop(x);
    E.label(skip);
    E.salu("s_mov_b64 exec, -1");
  }

  // two's-complement negation of x (owned, in place) where mask m is set, to the width W
  void neg_where(std::vector<Limb>& x, const Mask& m, uint32_t W) {
    if (m.k == 1 && !m.ones) return;
    std::vector<Limb> z(x.size(), Lit(0));
    std::vector<Limb> ng = add_chain(z, x, (uint32_t)x.size(), true);
    mask_top(ng, W);
    for (size_t j = 0; j < x.size(); j++) {
      const Limb t = vreg(ng[j]);
      if (m.k == 1) E.valu("v_mov_b32_e32 " + VL(x[j]) + ", " + VL(t));
      else vsel(x[j], x[j], t, m);
      drop(t);
    }
    drop_all(ng);
  }
  // the sign of a width-W value (bit W-1) as a mask
  Mask sign_mask(const std::vector<Limb>& x, uint32_t W) {
    const Limb t = x[Lw(W) - 1];
    if (t.lit()) {
      Mask m;
      m.k = 1;
      m.ones = (t.v >> ((W - 1) & 31)) & 1u;
      return m;
    }
    const Limb b = fresh();
    E.valu("v_bfe_u32 " + VL(b) + ", " + VL(t) + ", " + std::to_string((W - 1) & 31) + ", 1");
    const Mask m = vcmp("ne", b, 0);
    drop(b);
    return m;
  }
  // SDIV / SREM / SMOD by the msb case split (bv_device.h bv_sdiv / bv_srem / bv_smod)
  std::vector<Limb> sdivrem(uint32_t op, const std::vector<Limb>& a_in, const std::vector<Limb>& b_in, uint32_t W) {
    const uint32_t La = Lw(W);
    std::vector<Limb> a = own(a_in, La), b = own(b_in, La);
    note("sdivrem:abs");
    const Mask ma = sign_mask(a, W), mb = sign_mask(b, W);
    std::vector<Limb> aa = own(a, La), bb = own(b, La);
    neg_where(aa, ma, W);
    neg_where(bb, mb, W);
    std::vector<Limb> q, r;
    udivrem(aa, bb, W, q, r);
    note("sdivrem:sign");
    drop_all(aa);
    drop_all(bb);
    std::vector<Limb> out;
    if (op == K_SDIV) {
      drop_all(r);
      const Mask x = mop("xor", ma, mb);
      neg_where(q, x, W);
      E.srelease(x);
      out = q;
    } else if (op == K_SREM) {
      drop_all(q);
      neg_where(r, ma, W);
      out = r;
    } else {
      // SMOD: u = |a| urem |b|; u == 0 or both non-negative: u; a < 0 <= b: b - u;
      // a >= 0 > b: u + b; both negative: -u
      drop_all(q);
      std::vector<std::pair<Limb, Limb>> zp;
      for (uint32_t j = 0; j < La; j++) zp.push_back({r[j], Lit(0)});
      const Mask uz = eq_mask(zp);
      std::vector<Limb> bmu = add_chain(b, r, La, true);  // b - u
      std::vector<Limb> upb = add_chain(r, b, La, false); // u + b
      mask_top(bmu, W);
      mask_top(upb, W);
      std::vector<Limb> nu(La, Lit(0));
      std::vector<Limb> negu = add_chain(nu, r, La, true);  // -u
      mask_top(negu, W);
      const Mask nmb = mnot(mb), nma = mnot(ma);
      const Mask c1 = mop("and", ma, nmb), c2 = mop("and", nma, mb), c3 = mop("and", ma, mb);
      for (uint32_t j = 0; j < La; j++) {
        for (auto pr : {std::make_pair(&bmu, c1), std::make_pair(&upb, c2), std::make_pair(&negu, c3)}) {
          if (pr.second.k == 1 && !pr.second.ones) continue;
          const Limb t = vreg((*pr.first)[j]);
          if (pr.second.k == 1) E.valu("v_mov_b32_e32 " + VL(r[j]) + ", " + VL(t));
          else vsel(r[j], r[j], t, pr.second);
          drop(t);
        }
      }
      // u == 0: 0 (r is zero then unless a case above changed it: restore zero)
      if (!(uz.k == 1 && !uz.ones))
        for (uint32_t j = 0; j < La; j++) {
          if (uz.k == 1) E.valu("v_mov_b32_e32 " + VL(r[j]) + ", 0");
          else vsel(r[j], r[j], Reg(6), uz);
        }
      for (const Mask& m : {uz, nmb, nma, c1, c2, c3}) E.srelease(m);
      drop_all(bmu);
      drop_all(upb);
      drop_all(negu);
      out = r;
    }
    E.srelease(ma);
    E.srelease(mb);
    drop_all(a);
    drop_all(b);
    return out;
  }

  // ---- EXP -----------------------------------------------------------------------------------
  // base^e mod 2^W, left-to-right over the exponent's 2-bit digits (bv_device.h bv_exp): the wave's
  // longest exponent (ballots) fixes the step count; the exponent is pre-shifted so its top digit
  // sits at the top; per step two squarings and, where some lane's digit is non-zero, a multiply
  // by base^{1,2,3} (selected per lane)
  std::vector<Limb> exp_var(const std::vector<Limb>& base_in, const std::vector<Limb>& e_in, uint32_t W) {
    CondScope cs_(*this);
    const uint32_t La = Lw(W), C = 32 * La;
    std::vector<Limb> base = own(base_in, La), ex = own(e_in, La);
    std::vector<Limb> r(La);
    for (uint32_t j = 0; j < La; j++) {
      r[j] = fresh();
      E.valu("v_mov_b32_e32 " + VL(r[j]) + ", " + (j ? "0" : "1"));
    }
    std::vector<Limb> b2 = sqr_lo(base, La), b3;
    {
      std::vector<Limb> t = mul_lo(b2, base, La);
      b3 = own(t, La);
      drop_all(t);
      std::vector<Limb> t2 = own(b2, La);
      drop_all(b2);
      b2 = t2;
    }
    const Limb el = bitlen(ex);
    const int sD = sreg();
    wave_max(el, 9, sD);
    drop(el);
    // digits D = ceil(T / 2); ex <<= C - 2 D
    E.salu("s_add_u32 " + S(sD) + ", " + S(sD) + ", 1", {sD});
    E.salu("s_lshr_b32 " + S(sD) + ", " + S(sD) + ", 1", {sD});
    {
      const Limb sh = fresh();
      E.salu("s_lshl_b32 s41, " + S(sD) + ", 1", {41});
      E.salu("s_sub_u32 s41, " + imm(C) + ", s41", {41});
      E.valu("v_mov_b32_e32 " + VL(sh) + ", s41", {41});
      shift_limbs(ex, sh, true, Reg(6));
      drop(sh);
    }
    const std::string loop = E.newlab(), end = E.newlab();
    const Mask nz = mask_new();
    E.label(loop);
    E.salu("s_cmp_eq_u32 " + S(sD) + ", 0");
    E.ctl("s_cbranch_scc1 " + end);
    const Limb dg = fresh();
    E.valu("v_lshrrev_b32_e32 " + VL(dg) + ", 30, " + VL(ex[La - 1]));
    for (int i = (int)La - 1; i > 0; i--)
      E.valu("v_alignbit_b32 " + VL(ex[i]) + ", " + VL(ex[i]) + ", " + VL(ex[i - 1]) + ", 30");
    E.valu("v_lshlrev_b32_e32 " + VL(ex[0]) + ", 2, " + VL(ex[0]));
    for (int sq = 0; sq < 2; sq++) {
      std::vector<Limb> t = sqr_lo(r, La);
      assign(r, t);
    }
    {
      const std::string skip = E.newlab();
      E.valu("v_cmp_ne_u32_e64 " + SP(nz.s) + ", 0, " + VL(dg), {}, {nz.s, nz.s + 1});
      E.salu("s_cmp_eq_u64 " + SP(nz.s) + ", 0");
      E.ctl("s_cbranch_scc1 " + skip);
      const Mask m1 = vcmp("eq", dg, 1), m2 = vcmp("eq", dg, 2);
      std::vector<Limb> f(La);
      for (uint32_t j = 0; j < La; j++) {
        f[j] = fresh();
        vsel(f[j], b3[j], b2[j], m2);
        vsel(f[j], f[j], base[j], m1);
      }
      E.srelease(m1);
      E.srelease(m2);
      std::vector<Limb> p = mul_lo(r, f, La);
      drop_all(f);
      for (uint32_t j = 0; j < La; j++) {
        const Limb t = vreg(p[j]);
        vsel(r[j], r[j], t, nz);
        drop(t);
      }
      drop_all(p);
      E.label(skip);
    }
    drop(dg);
    E.salu("s_add_u32 " + S(sD) + ", " + S(sD) + ", -1", {sD});
    E.ctl("s_branch " + loop);
    E.label(end);
    E.srelease(nz);
    sfree(sD);
    drop_all(base);
    drop_all(ex);
    drop_all(b2);
    drop_all(b3);
    mask_top(r, W);
    return r;
  }

  // ---- Keccak-256 ----------------------------------------------------------------------------
  // keccak256 of the big-endian bytes of a width-w value (nbytes of them, pad10*1, rate 136 B),
  // as keccak_value (jit_device.h) and oracle/bveval.c vkeccak.  State: 25 lanes as (lo, hi)
  // VGPR halves; the permutation is a loop over rounds in three unrolled chunks of eight (the
  // round constants built on the SALU from a packed 7-bit code per round); rho and pi rotate each
  // lane into its destination in place along the pi cycle (one saved lane), chi keeps two saved
  // lanes per row
  static uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
  void keccak_f1600(std::vector<Limb>& st) {  // st: 50 owned registers, lane i = (st[2i], st[2i+1])
    CondScope cs_(*this);
    static const uint64_t RC[24] = {
        0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
        0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
        0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
        0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
        0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
        0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
    static const uint32_t kPos[7] = {0, 1, 3, 7, 15, 31, 63};
    auto lo = [&](int i) { return st[2 * i]; };
    auto hi = [&](int i) { return st[2 * i + 1]; };
    const int sT = sreg(), sK = sreg(), sR = sreg();  // packed table (pair), round count, RC lo/hi
    std::vector<Limb> c(10), rr(10);
    for (auto& x : c) x = fresh();
    for (auto& x : rr) x = fresh();
    const Limb t0 = fresh(), t1 = fresh(), s0 = fresh(), s1 = fresh();
    // 24 rounds in one loop: the round constants as 7-bit codes, 8 rounds per packed table; tables
    // 0..2 in three SGPR pairs, the current one shifted by 7 bits per round and replaced by the next
    // every 8 rounds
    const int sT1 = sreg(), sT2 = sreg();
    const int tabs[3] = {sT, sT1, sT2};
    for (int chunk = 0; chunk < 3; chunk++) {
      // 8 rounds x 7 bits: bit j of round k's code is RC bit kPos[j]
      uint64_t packed = 0;
      for (int k = 0; k < 8; k++) {
        uint64_t code = 0, back = 0;
        for (int j = 0; j < 7; j++) code |= ((RC[8 * chunk + k] >> kPos[j]) & 1ull) << j;
        for (int j = 0; j < 7; j++) back |= ((code >> j) & 1ull) << kPos[j];
        if (back != RC[8 * chunk + k]) fail("internal: a Keccak round constant outside the 7-bit code");
        packed |= code << (7 * k);
      }
      const int T = tabs[chunk];
      E.salu("s_mov_b32 " + S(T) + ", " + hexs((uint32_t)packed), {T});
      E.salu("s_mov_b32 " + S(T + 1) + ", " + hexs((uint32_t)(packed >> 32)), {T + 1});
    }
    E.salu("s_mov_b32 " + S(sK) + ", 24", {sK});
    {
      const std::string loop = E.newlab();
      E.label(loop);
      // theta: C[x] = xor of column x; a[x,y] ^= C[x-1] ^ rot(C[x+1], 1)
      for (int x = 0; x < 5; x++)
        for (int h = 0; h < 2; h++) {
          auto L_ = [&](int i) { return h ? hi(i) : lo(i); };
          const Limb d = c[2 * x + h];
          E.valu("v_bitop3_b32 " + VL(d) + ", " + VL(L_(x)) + ", " + VL(L_(x + 5)) + ", " + VL(L_(x + 10)) + " bitop3:0x96");
          E.valu("v_bitop3_b32 " + VL(d) + ", " + VL(d) + ", " + VL(L_(x + 15)) + ", " + VL(L_(x + 20)) + " bitop3:0x96");
        }
      for (int x = 0; x < 5; x++) {
        E.valu("v_alignbit_b32 " + VL(rr[2 * x]) + ", " + VL(c[2 * x]) + ", " + VL(c[2 * x + 1]) + ", 31");
        E.valu("v_alignbit_b32 " + VL(rr[2 * x + 1]) + ", " + VL(c[2 * x + 1]) + ", " + VL(c[2 * x]) + ", 31");
      }
      for (int y = 0; y < 25; y += 5)
        for (int x = 0; x < 5; x++)
          for (int h = 0; h < 2; h++) {
            const Limb a = h ? hi(y + x) : lo(y + x);
            E.valu("v_bitop3_b32 " + VL(a) + ", " + VL(a) + ", " + VL(c[2 * ((x + 4) % 5) + h]) + ", " +
                   VL(rr[2 * ((x + 1) % 5) + h]) + " bitop3:0x96");
          }
      // rho + pi along the cycle 1 -> 10 -> 7 -> ... (dst = rot(src, r)), backwards in place
      static const int kCyc[24] = {10, 7, 11, 17, 18, 3, 5, 16, 8, 21, 24, 4, 15, 23, 19, 13, 12, 2, 20, 14, 22, 9, 6, 1};
      static const int kRot[24] = {1, 3, 6, 10, 15, 21, 28, 36, 45, 55, 2, 14, 27, 41, 56, 8, 25, 43, 62, 18, 39, 61, 20, 44};
      auto rot_into = [&](const Limb& dl, const Limb& dh, const Limb& sl, const Limb& sh, int n) {
        if (n < 32) {
          E.valu("v_alignbit_b32 " + VL(dl) + ", " + VL(sl) + ", " + VL(sh) + ", " + std::to_string(32 - n));
          E.valu("v_alignbit_b32 " + VL(dh) + ", " + VL(sh) + ", " + VL(sl) + ", " + std::to_string(32 - n));
        } else {
          E.valu("v_alignbit_b32 " + VL(dl) + ", " + VL(sh) + ", " + VL(sl) + ", " + std::to_string(64 - n));
          E.valu("v_alignbit_b32 " + VL(dh) + ", " + VL(sl) + ", " + VL(sh) + ", " + std::to_string(64 - n));
        }
      };
      // dst k = kCyc[k] receives rot(src k, kRot[k]) with src 0 = lane 1, src k = kCyc[k-1]
      E.valu("v_mov_b32_e32 " + VL(t0) + ", " + VL(lo(1)));
      E.valu("v_mov_b32_e32 " + VL(t1) + ", " + VL(hi(1)));
      for (int k = 23; k >= 1; k--) rot_into(lo(kCyc[k]), hi(kCyc[k]), lo(kCyc[k - 1]), hi(kCyc[k - 1]), kRot[k]);
      rot_into(lo(kCyc[0]), hi(kCyc[0]), t0, t1, kRot[0]);
      // chi per row: a[x] ^= ~a[x+1] & a[x+2]; b0, b1 saved
      for (int y = 0; y < 25; y += 5)
        for (int h = 0; h < 2; h++) {
          auto A = [&](int x) { return h ? hi(y + x) : lo(y + x); };
          E.valu("v_mov_b32_e32 " + VL(s0) + ", " + VL(A(0)));
          E.valu("v_mov_b32_e32 " + VL(s1) + ", " + VL(A(1)));
          E.valu("v_bitop3_b32 " + VL(A(0)) + ", " + VL(A(0)) + ", " + VL(A(1)) + ", " + VL(A(2)) + " bitop3:0xd2");
          E.valu("v_bitop3_b32 " + VL(A(1)) + ", " + VL(A(1)) + ", " + VL(A(2)) + ", " + VL(A(3)) + " bitop3:0xd2");
          E.valu("v_bitop3_b32 " + VL(A(2)) + ", " + VL(A(2)) + ", " + VL(A(3)) + ", " + VL(A(4)) + " bitop3:0xd2");
          E.valu("v_bitop3_b32 " + VL(A(3)) + ", " + VL(A(3)) + ", " + VL(A(4)) + ", " + VL(s0) + " bitop3:0xd2");
          E.valu("v_bitop3_b32 " + VL(A(4)) + ", " + VL(A(4)) + ", " + VL(s0) + ", " + VL(s1) + " bitop3:0xd2");
        }
      // iota: RC from the round's 7-bit code (bit j -> RC bit kPos[j])
      E.salu("s_and_b32 s40, " + S(sT) + ", 0x7f", {40});
      E.salu("s_and_b32 " + S(sR) + ", s40, 3", {sR});  // positions 0 and 1
      for (int j = 2; j < 6; j++) {
        E.salu("s_and_b32 s41, s40, " + imm(1u << j), {41});
        E.salu("s_lshl_b32 s41, s41, " + std::to_string(kPos[j] - j), {41});
        E.salu("s_or_b32 " + S(sR) + ", " + S(sR) + ", s41", {sR});
      }
      E.salu("s_and_b32 s41, s40, 64", {41});
      E.salu("s_lshl_b32 " + S(sR + 1) + ", s41, 25", {sR + 1});
      E.valu("v_xor_b32_e32 " + VL(lo(0)) + ", " + S(sR) + ", " + VL(lo(0)));
      E.valu("v_xor_b32_e32 " + VL(hi(0)) + ", " + S(sR + 1) + ", " + VL(hi(0)));
      E.salu("s_lshr_b64 " + SP(sT) + ", " + SP(sT) + ", 7", {sT, sT + 1});
      E.salu("s_add_u32 " + S(sK) + ", " + S(sK) + ", -1", {sK});
      // every 8 rounds the next table (s_cselect keeps SCC)
      E.salu("s_and_b32 s40, " + S(sK) + ", 7", {40});
      E.salu("s_cmp_eq_u32 s40, 0");
      E.salu("s_cselect_b64 " + SP(sT) + ", " + SP(sT1) + ", " + SP(sT), {sT, sT + 1});
      E.salu("s_cselect_b64 " + SP(sT1) + ", " + SP(sT2) + ", " + SP(sT1), {sT1, sT1 + 1});
      E.salu("s_cmp_lg_u32 " + S(sK) + ", 0");
      E.ctl("s_cbranch_scc1 " + loop);
    }
    sfree(sT1);
    sfree(sT2);
    drop_all(c);
    drop_all(rr);
    drop(t0);
    drop(t1);
    drop(s0);
    drop(s1);
    sfree(sT);
    sfree(sK);
    sfree(sR);
  }
  std::vector<Limb> keccak(const std::vector<Limb>& v, uint32_t w, uint32_t nbytes) {
    const uint32_t nblk = nbytes / 136 + 1;
    std::vector<Limb> st(50);
    // the big-endian chunk of the value starting at message byte m, as the little-endian word of
    // the sponge (bytes m .. m+3); bytes past the value are zero
    auto word_at = [&](uint32_t m) -> Limb {
      if (m >= nbytes) return Lit(0);
      const int64_t p = 8 * ((int64_t)nbytes - (int64_t)m - 4);  // value bit of the chunk's low byte
      Limb f;
      if (p >= 0) {
        f = bits(v, w, (uint32_t)p, 32);
      } else {
        const uint32_t nb = (uint32_t)(nbytes - m);  // 1..3 valid bytes, the chunk's top bytes
        const Limb g = bits(v, w, 0, 8 * nb);
        if (g.lit()) {
          f = Lit(g.v << (32 - 8 * nb));
        } else {
          f = fresh();
          E.valu("v_lshlrev_b32_e32 " + VL(f) + ", " + std::to_string(32 - 8 * nb) + ", " + VL(g));
        }
        drop(g);
      }
      if (f.lit()) return Lit(bswap32(f.v));
      const Limb d = fresh();
      E.salu("s_mov_b32 s41, 0x10203", {41});
      E.valu("v_perm_b32 " + VL(d) + ", " + VL(f) + ", " + VL(f) + ", s41", {41});
      drop(f);
      return d;
    };
    for (uint32_t blk = 0; blk < nblk; blk++) {
      for (uint32_t h = 0; h < 34; h++) {
        const uint32_t m = blk * 136 + 4 * h;
        Limb x = word_at(m);
        uint32_t pad = 0;
        for (uint32_t k = 0; k < 4; k++) {
          if (m + k == nbytes) pad |= 0x01u << (8 * k);
          if (m + k == nblk * 136 - 1) pad |= 0x80u << (8 * k);
        }
        if (pad) {
          if (x.lit()) {
            x = Lit(x.v ^ pad);
          } else {
            const Limb d = fresh();
            if (inl(pad)) E.valu("v_xor_b32_e32 " + VL(d) + ", " + imm(pad) + ", " + VL(x));
            else E.valu("v_xor_b32_e32 " + VL(d) + ", " + hexs(pad) + ", " + VL(x));
            drop(x);
            x = d;
          }
        }
        if (blk == 0) {
          st[h] = fresh();
          E.valu("v_mov_b32_e32 " + VL(st[h]) + ", " + src(x));
        } else if (!(x.lit() && x.v == 0)) {
          if (x.lit() && !inl(x.v)) E.valu("v_xor_b32_e32 " + VL(st[h]) + ", " + hexs(x.v) + ", " + VL(st[h]));
          else E.valu("v_xor_b32_e32 " + VL(st[h]) + ", " + src(x) + ", " + VL(st[h]));
        }
        drop(x);
      }
      if (blk == 0)
        for (uint32_t h = 34; h < 50; h++) {
          st[h] = fresh();
          E.valu("v_mov_b32_e32 " + VL(st[h]) + ", 0");
        }
      keccak_f1600(st);
    }
    // digest: value limb j = bswap(state half 7 - j)
    std::vector<Limb> out(8);
    E.salu("s_mov_b32 s41, 0x10203", {41});
    for (uint32_t j = 0; j < 8; j++) {
      out[j] = fresh();
      E.valu("v_perm_b32 " + VL(out[j]) + ", " + VL(st[7 - j]) + ", " + VL(st[7 - j]) + ", s41", {41});
    }
    drop_all(st);
    return out;
  }

  void emit(const Instr& in, size_t k, const std::string& next) {
    const uint32_t d = in.dst, W = in.wd, Ld = Lw(W);
    switch (in.op) {
      case K_CONST: {
        std::vector<Limb> r(Ld);
        for (uint32_t j = 0; j < Ld; j++) r[j] = Lit(P.consts[in.p0 + j]);
        if (W == 1) {
          Mask m;
          m.k = 1;
          m.ones = P.consts[in.p0] & 1u;
          val[d].m = m;
        }
        set(d, r);
        break;
      }
      case K_COORD: {
        if (eval_kernel) {
          set(d, soa_limbs(in, d));
          break;
        }
        std::vector<Limb> r = gen_value(in.p0, need[d]);
        set(d, r);
        cval[in.p0] = d;
        break;
      }
      case K_ADD: case K_SUB: case K_NEG: {
        const uint32_t n = std::min(Ld, demanded(d));
        std::vector<Limb> x = in.op == K_NEG ? std::vector<Limb>(n, Lit(0)) : limbs(in.a, n);
        std::vector<Limb> y = in.op == K_NEG ? limbs(in.a, n) : limbs(in.b, n);
        std::vector<Limb> r = add_chain(x, y, n, in.op != K_ADD);
        r.resize(Ld);
        if (n == Ld) mask_top(r, W);
        set(d, r);
        break;
      }
      case K_MUL: {
        {
          auto ms = mulshare.find({std::min(in.a, in.b), std::max(in.a, in.b)});
          if (ms != mulshare.end() && ms->second.size() == Ld) {  // an UMUL_NOOVF's product
            std::vector<Limb> r = ms->second;
            mulshare.erase(ms);
            mask_top(r, W);
            set(d, r);
            break;
          }
        }
        const uint32_t n = std::min(Ld, demanded(d));
        std::vector<Limb> a = limbs(in.a, n), b = limbs(in.b, n), acc(n, Lit(0));  // acc owns
        for (uint32_t i = 0; i < n; i++) {
          if (a[i].lit() && a[i].v == 0) continue;
          std::vector<Limb> lo(n, Lit(0)), hi(n, Lit(0));
          bool anyv = false;
          for (uint32_t j = 0; i + j < n; j++) {
            const Limb x = a[i], y = b[j];
            if (y.lit() && y.v == 0) continue;
            if (x.lit() && y.lit()) {
              const uint64_t p = (uint64_t)x.v * y.v;
              lo[i + j] = Lit((uint32_t)p);
              if (i + j + 1 < n) hi[i + j + 1] = Lit((uint32_t)(p >> 32));
              continue;
            }
            anyv = true;
            // VOP3: literal operands through s41 (one SGPR per instruction)
            const Limb vx = x.reg() ? x : y, ly = x.reg() ? y : x;
            std::string so;
            // a literal operand goes through s41 (read by the multiplies: an SGPR the hazard table
            // tracks; a temporary initializer_list here would dangle)
            const bool via_s41 = ly.lit() && !inl(ly.v);
            if (via_s41) {
              E.salu("s_mov_b32 s41, " + hexs(ly.v), {41});
              so = "s41";
            } else {
              so = src(ly);
            }
            Limb dl, dh;
            product(vx, so, via_s41, true, i + j + 1 < n, dl, dh);
            lo[i + j] = dl;
            if (i + j + 1 < n) hi[i + j + 1] = dh;
          }
          (void)anyv;
          std::vector<Limb> s1 = add_chain(acc, lo, n, false);
          for (auto& t : acc) drop(t);
          for (auto& t : lo) drop(t);
          std::vector<Limb> s2 = add_chain(s1, hi, n, false);
          for (auto& t : s1) drop(t);
          for (auto& t : hi) drop(t);
          acc = s2;
        }
        acc.resize(Ld);
        if (n == Ld) mask_top(acc, W);
        set(d, acc);
        break;
      }
      case K_UMUL_NOOVF: {
        // the full 2La-limb product (schoolbook; zero literal limbs skipped: LASER's overflow checks
        // multiply a small count by a word), then "no bit at or above wa" as one zero test.  A MUL of
        // the same operands later in the program (batchOverflow: require(cnt * value / cnt == value)
        // next to amount = cnt * value) takes the product's low limbs from here (mulshare)
        const uint32_t wa = in.p1, La = Lw(wa), n = 2 * La;
        const auto mk = std::make_tuple(std::min(in.a, in.b), std::max(in.a, in.b), wa);
        auto mi = mul_at.find(mk);
        const bool share = !cond && !no_mulshare() && mi != mul_at.end() && mi->second > k;
        std::vector<Limb> a = limbs(in.a, La), b = limbs(in.b, La), acc(n, Lit(0));  // acc owns
        for (uint32_t i = 0; i < La; i++) {
          if (a[i].lit() && a[i].v == 0) continue;
          std::vector<Limb> lo(n, Lit(0)), hi(n, Lit(0));
          for (uint32_t j = 0; j < La; j++) {
            const Limb x = a[i], y = b[j];
            if (y.lit() && y.v == 0) continue;
            if (x.lit() && y.lit()) {
              const uint64_t p = (uint64_t)x.v * y.v;
              lo[i + j] = Lit((uint32_t)p);
              hi[i + j + 1] = Lit((uint32_t)(p >> 32));
              continue;
            }
            const Limb vx = x.reg() ? x : y, ly = x.reg() ? y : x;
            std::string so;
            const bool via_s41 = ly.lit() && !inl(ly.v);
            if (via_s41) {
              E.salu("s_mov_b32 s41, " + hexs(ly.v), {41});
              so = "s41";
            } else {
              so = src(ly);
            }
            // the product's limb 0 is the low half of a0 * b0 alone: it carries nothing into the limbs
            // the test reads (at or above wa >= 32), so it is not computed
            const bool lo_dead = i + j == 0 && wa >= 32 && !share;
            Limb dl = Lit(0), dh;
            product(vx, so, via_s41, !lo_dead, true, dl, dh);
            lo[i + j] = dl;
            hi[i + j + 1] = dh;
          }
          std::vector<Limb> s1 = add_chain(acc, lo, n, false);
          for (auto& t : acc) drop(t);
          for (auto& t : lo) drop(t);
          std::vector<Limb> s2 = add_chain(s1, hi, n, false);
          for (auto& t : s1) drop(t);
          for (auto& t : hi) drop(t);
          acc = s2;
        }
        std::vector<std::pair<Limb, Limb>> prs;
        std::vector<Limb> tmp;  // owned
        for (uint32_t q = 0; q < n; q++) {
          const uint32_t bit0 = 32 * q;
          const uint32_t m = bit0 + 32 <= wa ? 0u : (bit0 >= wa ? 0xFFFFFFFFu : ~((1u << (wa - bit0)) - 1u));
          if (!m) continue;
          if (acc[q].lit()) {
            prs.push_back({Lit(acc[q].v & m), Lit(0)});
          } else if (m == 0xFFFFFFFFu) {
            prs.push_back({acc[q], Lit(0)});
          } else {
            const Limb t = and_lit(acc[q], m);
            tmp.push_back(t);
            prs.push_back({t, Lit(0)});
          }
        }
        set_mask(d, eq_mask(prs));
        for (auto& t : tmp) drop(t);
        if (share) {
          std::vector<Limb> low(acc.begin(), acc.begin() + La);  // the references move to mulshare
          for (uint32_t q = La; q < n; q++) drop(acc[q]);
          auto& slot = mulshare[{std::min(in.a, in.b), std::max(in.a, in.b)}];
          for (auto& t : slot) drop(t);
          slot = low;
        } else {
          for (auto& t : acc) drop(t);
        }
        break;
      }
      case K_SHL: case K_LSHR: case K_ASHR: {
        if (!need[d]) {
          set(d, std::vector<Limb>(Ld));
          break;
        }
        std::vector<Limb> r = shift_var(in.op, limbs(in.a, Ld), in.b, W);
        set(d, r);
        break;
      }
      case K_SDIV: case K_SREM: case K_SMOD: {
        if (!need[d]) {
          set(d, std::vector<Limb>(Ld));
          break;
        }
        set(d, sdivrem(in.op, limbs(in.a, Ld), limbs(in.b, Ld), W));
        break;
      }
      case K_EXP: {
        if (!need[d]) {
          set(d, std::vector<Limb>(Ld));
          break;
        }
        set(d, exp_var(limbs(in.a, Ld), limbs(in.b, Ld), W));
        break;
      }
      case K_KECCAK: {
        if (!need[d]) {
          set(d, std::vector<Limb>(Ld));
          break;
        }
        set(d, keccak(in.a == MG_NONE ? std::vector<Limb>() : limbs(in.a, L(in.a)),
                      in.a == MG_NONE ? 0u : P.vwidth[in.a], in.p0));
        break;
      }
      case K_UDIV: case K_UREM: {
        if (!need[d]) {
          set(d, std::vector<Limb>(Ld));
          break;
        }
        if (!lit_divisor(in.b, Ld)) {
          std::vector<Limb> q, r;
          udivrem(limbs(in.a, Ld), limbs(in.b, Ld), W, q, r);
          if (in.op == K_UDIV) {
            drop_all(r);
            set(d, q);
          } else {
            drop_all(q);
            set(d, r);
          }
          break;
        }
        const uint32_t dv = P.consts[def_of(in.b)->p0];
        std::vector<Limb> x = limbs(in.a, Ld), r(Ld, Lit(0));
        if (dv == 0) {  // SMT-LIB: x / 0 = ~0 (to the width), x % 0 = x
          for (uint32_t j = 0; j < Ld; j++) {
            if (in.op == K_UDIV) r[j] = Lit(j == Ld - 1 ? topmask(W) : 0xFFFFFFFFu);
            else { r[j] = x[j]; E.retain(r[j]); }
          }
          set(d, r);
          break;
        }
        // normalised divisor dn = dv << s (top bit set) and its reciprocal v = (2^64 - 1) / dn - 2^32;
        // the dividend shifted by s into Ld + 1 limbs; then one Moller-Granlund 2/1 step per limb
        const uint32_t sh = (uint32_t)__builtin_clz(dv), dn = dv << sh;
        const uint32_t rv = (uint32_t)(~0ull / dn - (1ull << 32));
        std::vector<Limb> xs(Ld + 1);
        for (uint32_t j = 0; j <= Ld; j++) {
          const Limb hi = j < Ld ? x[j] : Lit(0), lo = j ? x[j - 1] : Lit(0);
          if (sh == 0) {
            xs[j] = hi;
            E.retain(hi);
          } else {
            xs[j] = bits(std::vector<Limb>{lo, hi}, 64, 32 - sh, 32);
          }
        }
        Limb rem = xs[Ld];  // < 2^sh <= dn: the first step's high word
        E.salu("s_mov_b32 s40, " + hexs(dn), {40});
        E.salu("s_mov_b32 s41, " + hexs(rv), {41});
        Mask mk;
        mk.k = 2;
        mk.s = E.salloc();
        const std::string M = SP(mk.s);
        for (int32_t j = (int32_t)Ld - 1; j >= 0; j--) {
          const Limb u1 = vreg(rem), u0 = vreg(xs[j]);
          drop(rem);
          drop(xs[j]);
          const Limb q0 = fresh(), q1 = fresh(), t = fresh(), rr = fresh();
          // (q1:q0) = rv * u1 + (u1 + 1 : u0)
          E.valu("v_mul_lo_u32 " + VL(q0) + ", " + VL(u1) + ", s41", {41});
          E.valu("v_mul_hi_u32 " + VL(q1) + ", " + VL(u1) + ", s41", {41});
          E.valu("v_add_co_u32_e32 " + VL(q0) + ", vcc, " + VL(q0) + ", " + VL(u0), {}, {kVCC, kVCC + 1});
          E.valu("v_addc_co_u32_e32 " + VL(q1) + ", vcc, " + VL(q1) + ", " + VL(u1) + ", vcc", {kVCC, kVCC + 1},
                 {kVCC, kVCC + 1});
          E.valu("v_add_u32_e32 " + VL(q1) + ", 1, " + VL(q1));
          // r = u0 - q1 * dn (mod 2^32)
          E.valu("v_mul_lo_u32 " + VL(t) + ", " + VL(q1) + ", s40", {40});
          E.valu("v_sub_u32_e32 " + VL(rr) + ", " + VL(u0) + ", " + VL(t));
          // r > q0: q1 - 1, r + dn
          E.valu("v_cmp_gt_u32_e64 " + M + ", " + VL(rr) + ", " + VL(q0), {}, {mk.s, mk.s + 1});
          E.valu("v_add_u32_e32 " + VL(t) + ", -1, " + VL(q1));
          E.valu("v_add_u32_e32 " + VL(q0) + ", s40, " + VL(rr), {40});
          E.valu("v_cndmask_b32_e64 " + VL(q1) + ", " + VL(q1) + ", " + VL(t) + ", " + M, {mk.s, mk.s + 1});
          E.valu("v_cndmask_b32_e64 " + VL(rr) + ", " + VL(rr) + ", " + VL(q0) + ", " + M, {mk.s, mk.s + 1});
          // r >= dn: q1 + 1, r - dn
          E.valu("v_cmp_le_u32_e64 " + M + ", s40, " + VL(rr), {40}, {mk.s, mk.s + 1});
          E.valu("v_add_u32_e32 " + VL(t) + ", 1, " + VL(q1));
          E.valu("v_subrev_u32_e32 " + VL(q0) + ", s40, " + VL(rr), {40});
          E.valu("v_cndmask_b32_e64 " + VL(q1) + ", " + VL(q1) + ", " + VL(t) + ", " + M, {mk.s, mk.s + 1});
          E.valu("v_cndmask_b32_e64 " + VL(rr) + ", " + VL(rr) + ", " + VL(q0) + ", " + M, {mk.s, mk.s + 1});
          drop(u1);
          drop(u0);
          drop(q0);
          drop(t);
          if (in.op == K_UDIV) r[j] = q1;
          else drop(q1);
          rem = rr;
        }
        E.srelease(mk);
        if (in.op == K_UREM) {
          if (sh) {
            const Limb d0 = fresh();
            E.valu("v_lshrrev_b32_e32 " + VL(d0) + ", " + std::to_string(sh) + ", " + VL(rem));
            drop(rem);
            rem = d0;
          }
          r[0] = rem;
        } else {
          drop(rem);
        }
        set(d, r);
        break;
      }
      case K_AND: case K_OR: case K_XOR: {
        if (W == 1) {
          const char* op = in.op == K_AND ? "and" : in.op == K_OR ? "or" : "xor";
          set_mask(d, mop(op, mask_of(in.a), mask_of(in.b)));
          break;
        }
        std::vector<Limb> r(Ld);
        for (uint32_t j = 0; j < Ld; j++) {
          if (!(need[d] >> j & 1)) continue;
          const Limb a = limb(in.a, j), b = limb(in.b, j);
          if (a.lit() && b.lit()) {
            r[j] = Lit(in.op == K_AND ? (a.v & b.v) : in.op == K_OR ? (a.v | b.v) : (a.v ^ b.v));
            continue;
          }
          const Limb l = a.lit() ? a : b, v = a.lit() ? b : a;
          if (l.lit()) {
            if ((in.op == K_AND && l.v == 0xFFFFFFFFu) || (in.op != K_AND && l.v == 0)) {
              E.retain(v);
              r[j] = v;
              continue;
            }
            if (in.op == K_AND && l.v == 0) { r[j] = Lit(0); continue; }
            if (in.op == K_OR && l.v == 0xFFFFFFFFu) { r[j] = Lit(0xFFFFFFFFu); continue; }
          }
          if (in.op != K_XOR && a == b) {
            E.retain(a);
            r[j] = a;
            continue;
          }
          const char* op = in.op == K_AND ? "v_and_b32_e32 " : in.op == K_OR ? "v_or_b32_e32 " : "v_xor_b32_e32 ";
          const Limb dd = fresh();
          E.valu(op + VL(dd) + ", " + src(l.lit() ? l : a) + ", " + VL(l.lit() ? v : b));
          r[j] = dd;
        }
        set(d, r);
        break;
      }
      case K_NOT: {
        if (W == 1) {
          set_mask(d, mnot(mask_of(in.a)));
          break;
        }
        std::vector<Limb> r(Ld);
        for (uint32_t j = 0; j < Ld; j++) {
          if (!(need[d] >> j & 1)) continue;
          const Limb a = limb(in.a, j);
          if (a.lit()) {
            r[j] = Lit(~a.v);
            continue;
          }
          const Limb dd = fresh();
          E.valu("v_not_b32_e32 " + VL(dd) + ", " + VL(a));
          r[j] = dd;
        }
        mask_top(r, W);
        set(d, r);
        break;
      }
      case K_COPY: {
        if (W == 1 && val[in.a].m.k) {
          E.sretain(val[in.a].m);
          val[d].m = val[in.a].m;
        }
        if (is_spilled(in.a)) reload(in.a);
        std::vector<Limb> r = val[in.a].l;
        for (auto& x : r) E.retain(x);
        set(d, r);
        break;
      }
      case K_ITE: {
        const Mask c = mask_of(in.a);
        if (W == 1) {
          if (c.k == 1) {
            const Mask x = mask_of(c.ones ? in.b : in.c);
            E.sretain(x);
            set_mask(d, x);
            break;
          }
          // (c & b) | (e & ~c): the else side in one s_andn2_b64 (a literal else folds)
          const Mask t = mop("and", c, mask_of(in.b));
          const Mask e = mask_of(in.c);
          Mask f;
          if (e.k == 1) {
            if (e.ones) {
              f = mnot(c);
            } else {
              f.k = 1;
              f.ones = false;
            }
          } else {
            f = mop_andn(e, c);
          }
          set_mask(d, mop("or", t, f));
          E.srelease(t);
          E.srelease(f);
          break;
        }
        std::vector<Limb> r(Ld);
        if (c.k == 1) {
          for (uint32_t j = 0; j < Ld; j++) {
            if (!(need[d] >> j & 1)) continue;
            r[j] = limb(c.ones ? in.b : in.c, j);
            E.retain(r[j]);
          }
          set(d, r);
          break;
        }
        if (c.k == 2 && !no_ite_e64() && !E.fresh_valu_write(c.s)) {  // the mask straight from its SGPR pair
          for (uint32_t j = 0; j < Ld; j++) {
            if (!(need[d] >> j & 1)) continue;
            r[j] = sel_mask(limb(in.b, j), limb(in.c, j), c);
          }
          set(d, r);
          break;
        }
        mask_to_vcc(c);
        for (uint32_t j = 0; j < Ld; j++) {
          if (!(need[d] >> j & 1)) continue;
          r[j] = sel(limb(in.b, j), limb(in.c, j));
        }
        set(d, r);
        break;
      }
      case K_EQ: {
        const uint32_t La = Lw(in.p1);
        if (in.p1 == 1) {
          set_mask(d, mnot_xor(mask_of(in.a), mask_of(in.b)));
          break;
        }
        set_mask(d, no_eq_cache() ? [&] {
          std::vector<std::pair<Limb, Limb>> prs;
          for (uint32_t j = 0; j < La; j++) prs.push_back({limb(in.a, j), limb(in.b, j)});
          return eq_mask(prs);
        }() : eq_ids(in.a, in.b, La));
        break;
      }
      case K_ULT: case K_ULE: case K_SLT: case K_SLE: {
        const uint32_t La = Lw(in.p1);
        const bool sgn = in.op == K_SLT || in.op == K_SLE;
        if (in.p1 == 1) {
          // Bool compares: a < b unsigned = ~a & b ; signed: a (= -1) < b (= 0) = a & ~b
          const Mask a = mask_of(in.a), b = mask_of(in.b);
          Mask lt = sgn ? mop_andn(a, b) : mop_andn(b, a);
          if (in.op == K_ULE || in.op == K_SLE) {
            const Mask gt = sgn ? mop_andn(b, a) : mop_andn(a, b);
            const Mask le = mnot(gt);
            E.srelease(gt);
            E.srelease(lt);
            lt = le;
          }
          set_mask(d, lt);
          break;
        }
        slt_many = sgn && ((in.a < slt_lits.size() && slt_lits[in.a] >= 3) || (in.b < slt_lits.size() && slt_lits[in.b] >= 3));
        if (in.op == K_ULT || in.op == K_SLT) {
          set_mask(d, lt_mask(limbs(in.a, La), limbs(in.b, La), in.p1, sgn));
        } else {
          const Mask gt = lt_mask(limbs(in.b, La), limbs(in.a, La), in.p1, sgn);
          set_mask(d, mnot(gt));
          E.srelease(gt);
        }
        break;
      }
      case K_CONCAT: case K_EXTRACT: {  // limb by limb through field_of (operands may be views)
        std::vector<Limb> r(Ld);
        for (uint32_t j = 0; j < Ld; j++)
          if (need[d] >> j & 1) r[j] = field_of(in, 32 * j, std::min(32u, W - 32 * j));
        set(d, r);
        break;
      }
      case K_ZEXT: {
        const uint32_t La = Lw(in.p1);
        std::vector<Limb> r(Ld, Lit(0));
        for (uint32_t j = 0; j < La && j < Ld; j++) {
          if (!(need[d] >> j & 1)) continue;
          r[j] = limb(in.a, j);
          E.retain(r[j]);
        }
        set(d, r);
        break;
      }
      case K_SEXT: {
        const uint32_t wa = in.p1, La = Lw(wa);
        std::vector<Limb> r(Ld);
        for (uint32_t j = 0; j + 1 < La; j++) {
          if (!(need[d] >> j & 1)) continue;
          r[j] = limb(in.a, j);
          E.retain(r[j]);
        }
        const Limb t = limb(in.a, La - 1);
        Limb top, f;
        if (t.lit()) {
          const uint32_t s = (wa - 1) & 31;
          const int32_t x = (int32_t)(t.v << (31 - s)) >> (31 - s);
          top = Lit((uint32_t)x);
          f = Lit(x < 0 ? 0xFFFFFFFFu : 0u);
        } else {
          if (wa & 31) {
            top = fresh();
            E.valu("v_bfe_i32 " + VL(top) + ", " + VL(t) + ", 0, " + std::to_string(wa & 31));
          } else {
            top = t;
            E.retain(top);
          }
          f = fresh();
          E.valu("v_ashrrev_i32_e32 " + VL(f) + ", 31, " + VL(top));
        }
        r[La - 1] = top;
        for (uint32_t j = La; j < Ld; j++) {
          r[j] = f;
          E.retain(f);
        }
        drop(f);
        mask_top(r, W);
        set(d, r);
        break;
      }
      case K_LOOKUP: {
        const uint32_t Lk = Lw(in.b), n = in.c;
        auto key_test = [&](uint32_t kv) -> Mask {
          if (!no_eq_cache()) return eq_ids(in.a, kv, Lk);
          std::vector<std::pair<Limb, Limb>> prs;
          for (uint32_t j = 0; j < Lk; j++) prs.push_back({limb(in.a, j), limb(kv, j)});
          return eq_mask(prs);
        };
        if (in.wd == 1 && !no_bool_lookup()) {
          // a Bool lookup (the specialiser's compare pushdown): selects of lane masks on the scalar
          // unit, no limb materialised
          Mask cur = mask_of(in.p0);
          E.sretain(cur);
          for (int32_t p = (int32_t)n - 1; p >= 0; p--) {
            const uint32_t kv = P.vaux[in.p1 + 2 * p], vv = P.vaux[in.p1 + 2 * p + 1];
            const Mask h = key_test(kv);
            if (h.k == 1) {
              if (h.ones) {
                E.srelease(cur);
                cur = mask_of(vv);
                E.sretain(cur);
              }
              continue;
            }
            // nc = h ? v : cur = (h & v) | (cur & ~h), one SALU when either side is a literal (the first
            // select of the compare pushdown's chain meets its default 1: v | ~h, one s_orn2_b64)
            const Mask vm = mask_of(vv);
            Mask nc;
            if (cur.k == 1 && !cur.ones) {
              nc = mop("and", h, vm);
            } else if (cur.k == 1 && vm.k == 2) {
              nc.k = 2;
              nc.s = E.salloc();
              E.salu("s_orn2_b64 " + SP(nc.s) + ", " + SP(vm.s) + ", " + SP(h.s), {nc.s, nc.s + 1});
            } else if (cur.k == 1) {  // both literal, cur true: v ? 1 : ~h
              if (vm.ones) {
                nc.k = 1;
                nc.ones = true;
              } else {
                nc = mnot(h);
              }
            } else if (vm.k == 1) {
              nc = vm.ones ? mop("or", h, cur) : mop_andn(cur, h);
            } else {
              const Mask t = mop("and", h, vm);
              const Mask f = mop_andn(cur, h);
              nc = mop("or", t, f);
              E.srelease(t);
              E.srelease(f);
            }
            E.srelease(cur);
            E.srelease(h);
            cur = nc;
          }
          set_mask(d, cur);
          break;
        }
        // (the key tests and their run ORs stay in SGPR pairs over the limbs: only with room for them)
        if (n >= 2 && n <= 5 && !no_lookup_runs() && E.sfree() >= (int)(n + n * (n - 1) / 2 + 4)) {
          // The key tests first, then per limb the select chain with runs of priors holding the same
          // limb (a key's literal tail, a zero, the same register) merged into one select under the OR
          // of their tests: applied last to first, h_p ? v : (h_p-1 ? v : c) = (h_p | h_p-1) ? v : c.
          // (C4: the keccak preimage lookups' limbs are mostly such runs.)
          std::vector<Mask> hs;
          std::vector<uint32_t> ps;  // the priors left, in application order (last prior first)
          int base = -1;             // a prior that always matches: the chain starts at its value
          for (int32_t p = (int32_t)n - 1; p >= 0; p--) {
            const Mask h = key_test(P.vaux[in.p1 + 2 * p]);
            if (h.k == 1) {
              if (h.ones) {
                for (auto& m : hs) E.srelease(m);
                hs.clear();
                ps.clear();
                base = p;
              }
              continue;
            }
            hs.push_back(h);
            ps.push_back((uint32_t)p);
          }
          const uint32_t dflt = base >= 0 ? P.vaux[in.p1 + 2 * base + 1] : in.p0;
          std::map<std::pair<size_t, size_t>, Mask> ors;  // OR of hs[a..b]
          auto run_mask = [&](size_t a, size_t b) -> Mask {
            if (a == b) return hs[a];
            auto it = ors.find({a, b});
            if (it != ors.end()) return it->second;
            const Mask prev = b - 1 == a ? hs[a] : ors.at({a, b - 1});
            const Mask m = mop("or", prev, hs[b]);
            ors[{a, b}] = m;
            return m;
          };
          std::vector<Limb> res(Ld);
          for (uint32_t j = 0; j < Ld; j++) {
            if (!(need[d] >> j & 1)) continue;
            Limb c = limb(dflt, j);
            E.retain(c);
            for (size_t a = 0; a < ps.size();) {
              const Limb v = limb(P.vaux[in.p1 + 2 * ps[a] + 1], j);
              size_t b = a;
              while (b + 1 < ps.size() && limb(P.vaux[in.p1 + 2 * ps[b + 1] + 1], j) == v) b++;
              if (!(v == c)) {
                // run_mask memoises ORs; every run ending at b extends the one ending at b - 1
                for (size_t q = a + 1; q < b; q++) run_mask(a, q);
                const Mask m = run_mask(a, b);
                const Limb t = v3(v), f = v3(c);
                const Limb r = fresh();
                E.valu("v_cndmask_b32_e64 " + VL(r) + ", " + src(f) + ", " + src(t) + ", " + SP(m.s), {m.s, m.s + 1});
                drop(t);
                drop(f);
                drop(c);
                c = r;
              }
              a = b + 1;
            }
            res[j] = c;
          }
          for (auto& kv : ors) E.srelease(kv.second);
          for (auto& m : hs) E.srelease(m);
          set(d, res);
          break;
        }
        std::vector<Limb> cur(Ld);
        for (uint32_t j = 0; j < Ld; j++) {
          if (!(need[d] >> j & 1)) continue;
          cur[j] = limb(in.p0, j);
          E.retain(cur[j]);
        }
        for (int32_t p = (int32_t)n - 1; p >= 0; p--) {
          const uint32_t kv = P.vaux[in.p1 + 2 * p], vv = P.vaux[in.p1 + 2 * p + 1];
          Mask h;
          if (no_eq_cache()) {
            std::vector<std::pair<Limb, Limb>> prs;
            for (uint32_t j = 0; j < Lk; j++) prs.push_back({limb(in.a, j), limb(kv, j)});
            h = eq_mask(prs);
          } else {
            h = eq_ids(in.a, kv, Lk);
          }
          if (h.k == 1) {
            if (h.ones) {
              for (uint32_t j = 0; j < Ld; j++) {
                if (!(need[d] >> j & 1)) continue;
                drop(cur[j]);
                cur[j] = limb(vv, j);
                E.retain(cur[j]);
              }
            }
            continue;
          }
          mask_to_vcc(h);
          for (uint32_t j = 0; j < Ld; j++) {
            if (!(need[d] >> j & 1)) continue;
            const Limb s = sel(limb(vv, j), cur[j]);
            drop(cur[j]);
            cur[j] = s;
          }
          E.srelease(h);
        }
        set(d, cur);
        break;
      }
      case K_ASSERT: {
        litcache_clear();  // the next constraint's code starts; its literals are materialised anew
        const Mask m = mask_of(in.a);
        if (m.k == 1) {
          if (!m.ones) E.salu("s_mov_b64 s[38:39], 0", {38, 39});
        } else {
          E.salu("s_and_b64 s[38:39], s[38:39], " + SP(m.s), {38, 39});
        }
        bool later = false;  // the last ASSERT falls through to the group's end anyway
        for (size_t q = k + 1; q < code.size() && !later; q++) later = code[q].op == K_ASSERT;
        if (!gen_kernel && !eval_kernel && later) {
          // early exit: s[42:43] is ~0 when the launch does not stop early, so the OR is zero only
          // when every lane failed and the wave may leave
          E.salu("s_or_b64 s[40:41], s[38:39], s[42:43]", {40, 41});
          E.ctl("s_cbranch_scc0 " + next);
        }
        break;
      }
      case K_WATCH:
        if (eval_kernel) {
          CondScope cs_(*this);  // the stores are skipped without a watch buffer
          // watch row p0 + j of candidate i: watch + ((p0 + j) * n + i) * 4, in-range lanes only
          const uint32_t Lw_ = Lw(P.vwidth[in.a]);
          E.salu("s_cmp_eq_u64 s[12:13], 0");  // no watch buffer: nothing to store
          const std::string skip = E.newlab();
          E.ctl("s_cbranch_scc1 " + skip);
          E.salu("s_mov_b64 exec, s[24:25]");
          for (uint32_t j = 0; j < Lw_; j++) {
            const Limb x = vreg(limb(in.a, j));
            row_ptr(in.p0 + j, 12);
            E.mem("global_store_dword v8, " + VL(x) + ", s[40:41]");
            drop(x);
          }
          E.salu("s_mov_b64 exec, -1");
          E.label(skip);
        }
        break;
      default:
        fail("op " + std::to_string(in.op) + " outside the assembly tier");
    }
    (void)k;
  }
  Mask mnot_xor(const Mask& a, const Mask& b) {
    const Mask x = mop("xor", a, b);
    const Mask r = mnot(x);
    E.srelease(x);
    return r;
  }
  // a & ~b
  Mask mop_andn(const Mask& a, const Mask& b) {
    if (a.k == 2 && b.k == 2) {  // one s_andn2_b64
      Mask m;
      m.k = 2;
      m.s = E.salloc();
      E.salu("s_andn2_b64 " + SP(m.s) + ", " + SP(a.s) + ", " + SP(b.s), {m.s, m.s + 1});
      return m;
    }
    const Mask nb = mnot(b);
    const Mask r = mop("and", a, nb);
    E.srelease(nb);
    return r;
  }

  // MYTHGPU_JIT_ASM_NO_LDS_DEFER=1: wait for a dictionary's LDS reads right after them
  static bool no_lds_defer() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_LDS_DEFER");
      return g && g[0] == '1';
    }();
    return on;
  }
  // MYTHGPU_JIT_ASM_NO_GEN_WANT=1: every MIXED coordinate generated whole
  static bool no_gen_want() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_GEN_WANT");
      return g && g[0] == '1';
    }();
    return on;
  }
  // MYTHGPU_JIT_ASM_NO_LOOKUP_RUNS=1: a lookup's select chain one prior at a time
  static bool no_lookup_runs() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_LOOKUP_RUNS");
      return g && g[0] == '1';
    }();
    return on;
  }
  // MYTHGPU_JIT_ASM_NO_BOOL_LOOKUP=1: a Bool lookup selects limbs like any other
  static bool no_bool_lookup() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_BOOL_LOOKUP");
      return g && g[0] == '1';
    }();
    return on;
  }
  static bool no_eq_cache() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_NO_EQ_CACHE");
      return g && g[0] == '1';
    }();
    return on;
  }
  static bool gen_only() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_GEN_ONLY");
      return g && g[0] == '1';
    }();
    return on;
  }
  static bool debug_live() {
    static const bool on = getenv("MYTHGPU_JIT_ASM_DEBUG") != nullptr;
    return on;
  }
  // the values instruction `in` reads directly (a LOOKUP's prior keys excepted: each is pinned by its
  // key test only) and through the views it reads
  void operands_of(const Instr& in, size_t k, std::vector<uint32_t>& out) {
    std::function<void(uint32_t)> add = [&](uint32_t id) {
      if (id == MG_NONE || id >= val.size()) return;
      out.push_back(id);
      if (is_view(id)) {
        const Instr& vi = code[def[id]];
        add(vi.a);
        if (vi.op == K_CONCAT) add(vi.b);
      }
    };
    switch (in.op) {
      case K_CONST: break;
      case K_COORD: if (copysrc[k] != MG_NONE) add(copysrc[k]); break;
      case K_LOOKUP:
        add(in.a);
        add(in.p0);
        for (uint32_t q = 0; q < in.c; q++) add(P.vaux[in.p1 + 2 * q + 1]);
        break;
      default:
        add(in.a);
        if (in.op != K_NOT && in.op != K_NEG && in.op != K_EXTRACT && in.op != K_ZEXT && in.op != K_SEXT &&
            in.op != K_ASSERT && in.op != K_COPY && in.op != K_WATCH)
          add(in.b);
        if (in.op == K_ITE) add(in.c);
        break;
    }
  }
  void body(const std::string& next) {
    eqdiff.clear();  // a kernel abandoned midway (AsmFail: out of VGPRs at this depth) left its entries
    mulshare.clear();
    xcache.clear();
    xby.clear();
    hcache.clear();
    hby.clear();
    h_last.clear();
    litcache.clear();
    lit_last.clear();
    x_last.clear();
    eq_last.clear();
    dlimb.clear();
    E.on_free = [this](uint32_t g) {
      xcache_free(g);
      hcache_free(g);
      dlimb_free(g);
    };
    E.on_pressure = [this]() { return evict_one(); };
    E.on_hard = [this]() { return spill_one(); };
    spill_at.assign(val.size(), {});
    slot_busy.clear();
    pinned.clear();
    E.on_spressure = [this]() { return spill_mask(); };
    lvn_on = true;
    static const bool annotate = getenv("MYTHGPU_JIT_ASM_ANNOTATE") != nullptr;
    for (size_t k = 0; k < code.size(); k++) {
      const Instr& in = code[k];
      cur_k = k;
      if (is_view(in.dst)) continue;  // read through by its one reader (field_of)
      if (annotate)
        E.o << "  ; vcode " << k << " op " << in.op << " w " << in.wd << " dst " << in.dst << " a " << in.a << " b " << in.b
            << "\n";
      if (spill_on) {  // the values this instruction reads stay in registers while it is emitted
        pinned.clear();
        operands_of(in, k, pinned);
        for (size_t q = 0; q < pinned.size(); q++)
          if (is_spilled(pinned[q])) reload(pinned[q]);
      }
      emit(in, k, next);
      if (spill_on) pinned.clear();
      if (debug_live()) {
        int used = 0;
        for (int r = E.vfirst; r < 256; r++) used += E.vref[r] > 0;
        fprintf(stderr, "asm live %zu op %u w %u: %d VGPRs\n", k, in.op, in.wd, used);
        static const long at = getenv("MYTHGPU_JIT_ASM_DEBUG_AT") ? atol(getenv("MYTHGPU_JIT_ASM_DEBUG_AT")) : -1;
        if ((long)k == at) {
          std::map<uint32_t, int> byop;
          for (uint32_t id = 0; id < val.size(); id++) {
            if (!val[id].def) continue;
            int regs = 0;
            for (const auto& l : val[id].l) regs += l.reg();
            if (regs && def[id] >= 0) byop[code[def[id]].op] += regs;
          }
          for (const auto& kv : byop) fprintf(stderr, "  live from op %u: %d limbs\n", kv.first, kv.second);
        }
      }
      // values whose last reader is this instruction, and results nobody reads
      auto done = [&](uint32_t id) {
        if (id != MG_NONE && id < last.size() && last[id] <= (int32_t)k && val[id].def) {
          kill(id);
          val[id].def = false;
          if (!eqdiff.empty()) eq_forget(id);
        }
      };
      if (in.dst != MG_NONE && in.dst < last.size() && last[in.dst] < 0) done(in.dst);
      switch (in.op) {
        case K_CONST: break;
        case K_WATCH:
          if (eval_kernel) done(in.a);  // a value read last by its watch row store
          break;
        case K_COORD:
          if (copysrc[k] != MG_NONE) done(copysrc[k]);
          break;
        case K_LOOKUP:
          done(in.a);
          done(in.p0);
          for (uint32_t q = 0; q < 2 * in.c; q++) done(P.vaux[in.p1 + q]);
          break;
        default:
          done(in.a);
          if (in.b != MG_NONE) done(in.b);
          if (in.op == K_ITE) done(in.c);
          if (in.op == K_CONCAT || in.op == K_EXTRACT) {  // the operands of the views it read through
            std::function<void(uint32_t)> through = [&](uint32_t id) {
              if (!is_view(id)) return;
              const Instr& vi = code[def[id]];
              done(vi.a);
              through(vi.a);
              if (vi.op == K_CONCAT) {
                done(vi.b);
                through(vi.b);
              }
            };
            through(in.a);
            if (in.op == K_CONCAT) through(in.b);
          }
          break;
      }
    }
    for (auto& kv : mulshare)
      for (auto& t : kv.second) drop(t);
    mulshare.clear();
    for (auto& kv : eqdiff) drop(kv.second);  // values live to the end of the body
    eqdiff.clear();
    xcache_clear();
    litcache_clear();
    lvn_on = false;
    E.on_free = nullptr;
    E.on_pressure = nullptr;
    E.on_hard = nullptr;
    E.on_spressure = nullptr;
  }

  // ---------------------------------------------------------------------------------------
  // the kernel around the body
  // ---------------------------------------------------------------------------------------
  // The group key on the scalar unit per group (fmix64, 18 SALU, 8 of them multiplies) or from the VALU
  // table of the wave's next 64 groups (2 v_readlane per group + ~0.4 VALU amortised): the table pays
  // where the scalar unit is the busier one.  jit_asm_source decides per kernel from the first pass's
  // static SALU : VALU ratio (kSgkeyRatio); MYTHGPU_JIT_ASM_SGKEY=1 / =0 fixes the scalar / VALU key.
  // Measured (profiles/r06f_group_key_ab.jsonl, profiles/r06h_bench_*): C3 515 vs 482 G/s with the
  // table, C1 / etherstore / C4 +0.7-0.9 %, the C2 headline at 2^30 233 vs 229.6 with the scalar key.
  bool sgkey = false;
  static int sgkey_env() {
    static const int v = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_SGKEY");
      return g ? (g[0] == '1' ? 1 : 0) : -1;
    }();
    return v;
  }
  bool salu_group_key() const { return sgkey; }
  // 64-bit fmix64 of s[x:x+1] in place (SALU; s40/s41 scratch)
  void sfmix(int x) {
    auto xs = [&]() {
      E.salu("s_lshr_b32 s40, " + S(x + 1) + ", 1", {40});
      E.salu("s_xor_b32 " + S(x) + ", " + S(x) + ", s40", {x});
    };
    auto mul = [&](uint32_t clo, uint32_t chi) {
      E.salu("s_mul_hi_u32 s40, " + S(x) + ", " + hexs(clo), {40});
      E.salu("s_mul_i32 s41, " + S(x) + ", " + hexs(chi), {41});
      E.salu("s_add_u32 s40, s40, s41", {40});
      E.salu("s_mul_i32 s41, " + S(x + 1) + ", " + hexs(clo), {41});
      E.salu("s_add_u32 " + S(x + 1) + ", s40, s41", {x + 1});
      E.salu("s_mul_i32 " + S(x) + ", " + S(x) + ", " + hexs(clo), {x});
    };
    xs();
    mul(0xED558CCDu, 0xFF51AFD7u);
    xs();
    mul(0x1A85EC53u, 0xC4CEB9FEu);
    xs();
  }
  // per-lane fmix64 of v[lo], v[hi] in place (VALU; constants through s40/s41)
  void vfmix(int lo, int hi) {
    const Limb t1 = fresh(), t2 = fresh();
    auto xs = [&]() {
      E.valu("v_lshrrev_b32_e32 " + VL(t1) + ", 1, " + V(hi));
      E.valu("v_xor_b32_e32 " + V(lo) + ", " + V(lo) + ", " + VL(t1));
    };
    auto mul = [&](uint32_t clo, uint32_t chi) {
      E.salu("s_mov_b32 s40, " + hexs(clo), {40});
      E.salu("s_mov_b32 s41, " + hexs(chi), {41});
      E.valu("v_mul_hi_u32 " + VL(t1) + ", " + V(lo) + ", s40", {40});
      E.valu("v_mul_lo_u32 " + VL(t2) + ", " + V(lo) + ", s41", {41});
      E.valu("v_add_u32_e32 " + VL(t1) + ", " + VL(t1) + ", " + VL(t2));
      E.valu("v_mul_lo_u32 " + VL(t2) + ", " + V(hi) + ", s40", {40});
      E.valu("v_add_u32_e32 " + V(hi) + ", " + VL(t1) + ", " + VL(t2));
      E.valu("v_mul_lo_u32 " + V(lo) + ", " + V(lo) + ", s40", {40});
    };
    xs();
    mul(0xED558CCDu, 0xFF51AFD7u);
    xs();
    mul(0x1A85EC53u, 0xC4CEB9FEu);
    xs();
    drop(t1);
    drop(t2);
  }

  // ---------------------------------------------------------------------------------------
  // the eval kernel (mgj_eval): explicit coordinates from SoA rows [row][candidate] in HBM.
  // One candidate per lane (i < 2^30: 32-bit lane offsets), a grid-stride loop; the program's
  // coordinate rows are loaded in the order the program reads them, kPrefetch loads ahead of
  // their use (loads complete in order, so each use waits with vmcnt for exactly its row)
  // ---------------------------------------------------------------------------------------
  // loads kept in flight ahead of their use: MYTHGPU_JIT_ASM_PREFETCH fixes it (at most 60: vmcnt);
  // by default jit_asm_source sizes it to the registers the kernel's occupancy leaves (eval_depth)
  static uint32_t prefetch_env() {
    static const uint32_t n = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_PREFETCH");
      return g ? (uint32_t)std::max(1, std::min(60, atoi(g))) : 0u;
    }();
    return n;
  }
  uint32_t depth = 24;
  uint32_t prefetch_depth() const { return depth; }
  std::vector<uint32_t> rows;           // SoA rows in the order the program reads them
  std::vector<Limb> row_reg;            // registers of issued rows
  size_t rows_issued = 0, rows_used = 0;
  // Across groups: the first `ring` rows of the NEXT group are loaded into fixed registers (ring_reg,
  // held for the whole kernel) while this group's last rows are consumed, offsets in vnext, so the
  // queue never drains at a group boundary.  A ring row's value is copied out when consumed.
  // row_seq: issue position of each row among this iteration's loads (ring rows: before it, -ring..-1)
  std::vector<Limb> ring_reg;
  Limb vnext;
  // Tiled SoA (MG_JIT_SOA_TILED): candidate i's row r at ((i / 64) * coord_words + r) * 64 + i % 64 —
  // a group's rows are one contiguous block (C4: 243 x 256 B), so a wave's loads stay inside one
  // page (the row-major layout put them 4 n bytes apart: 7.7 % UTCL1 translation misses on C4)
  // and each row's address is the group base + an immediate.  s[26:27] this group's block, s[28:29]
  // the next group's (clamped to the last block)
  bool tiled = false;
  std::vector<long> row_seq;
  long loads = 0;

  // s[40:41] = base s[b:b+1] + row * n * 4 (n * 4 in s[20:21]: below 2^32, the first tier's eval kernel
  // takes n < 2^30, so s21 = 0 and one 32 x 32 -> 64 product is the whole offset)
  void row_ptr(uint32_t row, int b) {
    E.salu("s_mul_i32 s40, s20, " + hexs(row), {40});
    E.salu("s_mul_hi_u32 s41, s20, " + hexs(row), {41});
    E.salu("s_add_u32 s40, s40, " + S(b), {40});
    E.salu("s_addc_u32 s41, s41, " + S(b + 1), {41});
  }
  // Row-major loads keep the last loaded row's pointer (soa + row * n * 4, the same for every group) in
  // s[100:101]: the next row is one add away when it follows it (rows are mostly read in order), two
  // products and an add otherwise.  Valid until a label (a loop head or a join) is emitted.
  int64_t rp_row = -1;
  int rp_lab = -1;
  bool rp_used = false;
  void row_ptr_rm(uint32_t row) {
    const bool have = rp_row >= 0 && rp_lab == E.label_events;
    if (have && (int64_t)row == rp_row) {
    } else if (have && (int64_t)row == rp_row + 1) {
      E.salu("s_add_u32 s100, s100, s20", {100});
      E.salu("s_addc_u32 s101, s101, 0", {101});
    } else if (have && (int64_t)row > rp_row) {
      const uint32_t dl = (uint32_t)(row - rp_row);
      E.salu("s_mul_i32 s40, s20, " + hexs(dl), {40});
      E.salu("s_mul_hi_u32 s41, s20, " + hexs(dl), {41});
      E.salu("s_add_u32 s100, s100, s40", {100});
      E.salu("s_addc_u32 s101, s101, s41", {101});
    } else {
      E.salu("s_mul_i32 s100, s20, " + hexs(row), {100});
      E.salu("s_mul_hi_u32 s101, s20, " + hexs(row), {101});
      E.salu("s_add_u32 s100, s100, s4", {100});
      E.salu("s_addc_u32 s101, s101, s5", {101});
    }
    rp_row = row;
    rp_lab = E.label_events;
    rp_used = true;
  }
  // the load of SoA row `row` of the group whose block base is s[b:b+1] (tiled) or of the candidates
  // at offsets `voff` (row-major: s[4:5] + row * n * 4)
  // the 4-KiB page base of the last row loaded from each block (this group's in s[36:37], the next
  // group's in s[18:19]; -1: none): a row in the same page needs no address arithmetic
  int64_t page_at[2] = {-1, -1};
  void load_row(const Limb& d, uint32_t row, int b, const std::string& voff, const std::string& note) {
    if (tiled) {
      const uint64_t byte = (uint64_t)row * 256u, hi = byte & ~4095ull;
      std::string base = "s[" + std::to_string(b) + ":" + std::to_string(b + 1) + "]";
      if (hi) {
        const int w = b == 26 ? 0 : 1, pr = w ? 18 : 36;
        if (page_at[w] != (int64_t)hi) {
          E.salu("s_add_u32 " + S(pr) + ", " + S(b) + ", " + hexs((uint32_t)hi), {pr});
          E.salu("s_addc_u32 " + S(pr + 1) + ", " + S(b + 1) + ", 0", {pr + 1});
          page_at[w] = (int64_t)hi;
        }
        base = "s[" + std::to_string(pr) + ":" + std::to_string(pr + 1) + "]";
      }
      E.mem("global_load_dword " + VL(d) + ", v2, " + base + " offset:" + std::to_string(byte & 4095u) +
            "  ; soa row " + std::to_string(row) + note);
    } else {
      row_ptr_rm(row);
      E.mem("global_load_dword " + VL(d) + ", " + voff + ", s[100:101]  ; soa row " + std::to_string(row) + note);
    }
  }
  // s[d:d+1] = soa + g * coord_words * 256 for the group index in s[g]
  void block_base(int d, int g) {
    const uint32_t stride = P.coord_words * 256u;
    E.salu("s_mul_i32 " + S(d) + ", " + S(g) + ", " + hexs(stride), {d});
    E.salu("s_mul_hi_u32 " + S(d + 1) + ", " + S(g) + ", " + hexs(stride), {d + 1});
    E.salu("s_add_u32 " + S(d) + ", " + S(d) + ", s4", {d});
    E.salu("s_addc_u32 " + S(d + 1) + ", " + S(d + 1) + ", s5", {d + 1});
  }
  void issue_rows(size_t upto) {
    while (rows_issued < rows.size() && rows_issued < upto) {
      const Limb d = fresh();
      load_row(d, rows[rows_issued], 26, "v2", "");
      row_seq[rows_issued] = loads++;
      row_reg[rows_issued++] = d;
    }
  }
  // --- LDS-staged rows (tiled SoA): the row queue in LDS instead of VGPRs ---------------------
  // Each row is fetched by global_load_lds_dword (LDS-DMA: no VGPR while in flight) `gdepth` rows
  // ahead of its use into a per-wave LDS slot, and read into a VGPR by ds_read_b32 `sdepth` rows
  // ahead.  The queue's depth is then bounded by LDS (160 KiB per CU), not by the VGPRs the program
  // leaves: C4's program holds ~200 VGPRs (2 waves per SIMD), which left the register queue ~12
  // rows — 0.53 of HBM.  Slots: rows 0 .. D-1 of a group in slots 0 .. D-1 (the next group's are
  // fetched there while this group's last D rows are consumed), rows >= D in D+1 rotating slots
  // D + (p - D) % (D + 1): a slot is refilled only after the ds_read of its previous row was waited
  // for.  s34 = the wave's slot base, glds_v its LDS address per lane.
  bool glds = false;
  uint32_t gdepth = 0, sdepth = 4;
  Limb glds_v;
  size_t gl_issued = 0, staged = 0;
  long lgkm_n = 0;
  std::vector<long> gseq, lseq;  // VMEM / LGKM issue index of each row's glds / ds_read
  std::vector<Limb> stage_reg;
  // MYTHGPU_JIT_ASM_GLDS: 1 = the LDS queue where it is deeper than the register queue, N > 1 = the LDS
  // queue at depth N; unset / 0 = the register queue.  Opt-in: measured within +-3 % of the register
  // queue on C2 and C4 (profiles/r05i_eval_glds.jsonl) at ~2x its SALU and waits per row (M0, the
  // address pair, a vmcnt and an lgkmcnt wait), and the kernel is issue-bound
  // MYTHGPU_JIT_ASM_XCD=1: the eval kernel's XCD-aware block order (above; diagnostic until measured)
  static bool xcd_swizzle() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_XCD");
      return g && g[0] == '1';
    }();
    return on;
  }
  static bool glds_env() {
    static const bool on = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_GLDS");
      return g && g[0] && g[0] != '0';
    }();
    return on;
  }
  static uint32_t glds_fixed() {
    static const uint32_t n = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_GLDS");
      const int v = g ? atoi(g) : 0;
      return v > 1 ? (uint32_t)std::min(v, 60) : 0u;
    }();
    return n;
  }
  uint32_t glds_slot(size_t p) const { return p < gdepth ? (uint32_t)p : gdepth + (uint32_t)((p - gdepth) % (gdepth + 1)); }
  uint32_t glds_slots() const { return gdepth + (rows.size() > gdepth ? gdepth + 1 : 0); }
  // glds of row index idx: idx < M this group's row, else the next group's row idx - M
  void glds_issue(size_t idx) {
    const size_t M = rows.size();
    const bool next = idx >= M;
    const size_t p = next ? idx - M : idx;
    const int b = next ? 28 : 26;
    E.salu("s_add_u32 m0, s34, " + hexs(glds_slot(p) * 256u));
    const uint64_t byte = (uint64_t)rows[p] * 256u;
    std::string base = "s[" + std::to_string(b) + ":" + std::to_string(b + 1) + "]";
    if (byte) {
      E.salu("s_add_u32 s40, " + S(b) + ", " + hexs((uint32_t)byte), {40});
      E.salu("s_addc_u32 s41, " + S(b + 1) + ", 0", {41});
      base = "s[40:41]";
    } else {
      E.salu("s_nop 0");  // M0 -> LDS-DMA: one wait state
    }
    E.mem("global_load_lds_dword v2, " + base + "  ; soa row " + std::to_string(rows[p]) + (next ? " (next group)" : ""));
    if (!next) gseq[p] = loads;
    loads++;
  }
  void glds_upto(size_t u) {
    const size_t M = rows.size();
    while (gl_issued <= u && gl_issued < M + gdepth) glds_issue(gl_issued++);
  }
  void stage_upto(size_t u) {
    const size_t M = rows.size();
    while (staged <= u && staged < M) {
      const size_t t = staged++;
      const long after = loads - gseq[t] - 1;
      E.ctl("s_waitcnt vmcnt(" + std::to_string(std::min<long>(std::max<long>(after, 0), 63)) + ")");
      const Limb dv = fresh();
      E.mem("ds_read_b32 " + VL(dv) + ", " + VL(glds_v) + " offset:" + std::to_string(glds_slot(t) * 256u));
      lseq[t] = lgkm_n++;
      stage_reg[t] = dv;
    }
  }

  std::vector<Limb> soa_limbs(const Instr& in, uint32_t d) {
    const uint32_t Lc = Lw(in.wd);
    std::vector<Limb> r(Lc);
    for (uint32_t j = 0; j < Lc; j++) {
      if (!(need[d] >> j & 1)) continue;
      if (rows_used >= rows.size() || rows[rows_used] != in.p1 + j) fail("internal: SoA row order");
      if (glds) {
        const size_t p = rows_used++;
        stage_upto(p);
        E.ctl("s_waitcnt lgkmcnt(" + std::to_string(std::min<long>(std::max<long>(lgkm_n - lseq[p] - 1, 0), 15)) + ")");
        r[j] = stage_reg[p];
        stage_reg[p] = Limb{};
        glds_upto(p + gdepth);  // refills the slot row p - 1 (region 2) or row p + D - M (region 1) held
        stage_upto(p + sdepth);
        continue;
      }
      issue_rows(rows_used + 1);
      // loads return in order: wait until only the loads issued after this row are outstanding
      // (stores are not counted: the watch stores are conditional; an uncounted younger store only
      // makes the wait longer)
      const long after = loads - row_seq[rows_used] - 1;
      E.ctl("s_waitcnt vmcnt(" + std::to_string(std::min<long>(std::max<long>(after, 0), 63)) + ")");
      const size_t p = rows_used++;
      if (p < ring_reg.size()) {  // a ring register: copied out, reloaded for the next group below
        r[j] = fresh();
        E.valu("v_mov_b32_e32 " + VL(r[j]) + ", " + VL(ring_reg[p]));
      } else {
        r[j] = row_reg[p];
      }
      issue_rows(rows_used + prefetch_depth());  // keep that many loads in flight
      const size_t M = rows.size(), R = ring_reg.size();
      if (p + R >= M) {  // the next group's ring row p + R - M (clamped offsets: always in bounds)
        const size_t q = p + R - M;
        load_row(ring_reg[q], rows[q], 28, VL(vnext), " (next group)");
        loads++;
      }
    }
    return r;
  }

  std::string kernel_eval(const std::string& name) {
    E = Emitter();
    rp_row = -1;
    rp_lab = -1;
    rp_used = false;
    E.vhard = vhard;
    E.nlab = labels;
    E.vsoft = vsoft;
    census.clear();
    E.vfirst = kV0 + (int)pool.size();
    E.vhigh = E.vfirst;
    val.assign(P.vwidth.size(), Val{});
    rows.clear();
    for (const Instr& in : code)
      if (in.op == K_COORD)
        for (uint32_t j = 0; j < Lw(in.wd); j++)
          if (in.dst < need.size() && (need[in.dst] >> j & 1)) rows.push_back(in.p1 + j);
    row_reg.assign(rows.size(), Limb{});
    row_seq.assign(rows.size(), 0);
    glds = tiled && glds_env() && !rows.empty() && gdepth > 0 && !spill_on;
    if (glds) {
      gdepth = std::min<uint32_t>(gdepth, (uint32_t)rows.size());
      gseq.assign(rows.size(), 0);
      lseq.assign(rows.size(), 0);
      stage_reg.assign(rows.size(), Limb{});
    }
    auto& o = E.o;
    o << "  .text\n  .globl " << name << "\n  .p2align 8\n  .type " << name << ",@function\n" << name << ":\n";
    // arguments (soa, n, verdict_out, watch, nblk): s[4:5] soa, s[8:9] n, s[10:11] verdict, s[12:13] watch, s14 nblk
    E.ctl("s_load_dwordx2 s[4:5], s[0:1], 0x0");
    E.ctl("s_load_dwordx8 s[8:15], s[0:1], 0x8");
    E.valu("v_and_b32_e32 v1, 63, v0");
    E.valu("v_mov_b32_e32 v6, 0");
    E.valu("v_readfirstlane_b32 s3, v0", {}, {3});
    E.salu("s_lshr_b32 s3, s3, 6", {3});
    E.ctl("s_waitcnt lgkmcnt(0)");
    for (const auto& kv : pool) E.valu("v_mov_b32_e32 " + V((uint32_t)kv.second) + ", " + imm(kv.first));
    // n * 4 (64-bit) in s[20:21]; the wave's first candidate s16 = block * 256 + wave * 64; stride s17.
    // Solo: waves 1..3 leave at once and wave 0 evaluates the ONE group s16 = block * 64 — no group
    // loop: a solo kernel is tens of thousands of instructions (VMTests' expXY: 58 k), past the +-128 KiB
    // a branch reaches — so the engine launches ceil(n / 64) blocks for it (mgj_meta_eval_cpb below,
    // read by code_object_info); lanes past n store nothing, as in the loop
    E.salu("s_lshl_b64 s[20:21], s[8:9], 2", {20, 21});
    if (solo) {
      const std::string go = E.newlab();
      E.salu("s_cmp_eq_u32 s3, 0");
      E.ctl("s_cbranch_scc1 " + go);
      E.ctl("s_endpgm");
      E.label(go);
      E.salu("s_lshl_b32 s16, s2, 6", {16});
      E.salu("s_mov_b32 s17, 64", {17});
    } else if (xcd_swizzle()) {
      // blocks b and b + 8 share an XCD (MI355X_MICROARCH.md): with the block count a multiple of 8,
      // block b takes candidates at (b % 8) * (nblk / 8) + b / 8, so the blocks of one XCD sweep one
      // contiguous stretch of every SoA row (a bijection; otherwise the identity)
      const std::string keep = E.newlab();
      E.salu("s_mov_b32 s40, s2", {40});
      E.salu("s_and_b32 s41, s14, 7", {41});
      E.salu("s_cmp_eq_u32 s41, 0");
      E.ctl("s_cbranch_scc0 " + keep);
      E.salu("s_lshr_b32 s41, s14, 3", {41});
      E.salu("s_and_b32 s40, s2, 7", {40});
      E.salu("s_mul_i32 s40, s40, s41", {40});
      E.salu("s_lshr_b32 s41, s2, 3", {41});
      E.salu("s_add_u32 s40, s40, s41", {40});
      E.label(keep);
      E.salu("s_lshl_b32 s16, s40, 8", {16});
      E.salu("s_lshl_b32 s22, s3, 6", {22});
      E.salu("s_add_u32 s16, s16, s22", {16});
      E.salu("s_lshl_b32 s17, s14, 8", {17});
    } else {
      E.salu("s_lshl_b32 s16, s2, 8", {16});
      E.salu("s_lshl_b32 s22, s3, 6", {22});
      E.salu("s_add_u32 s16, s16, s22", {16});
      E.salu("s_lshl_b32 s17, s14, 8", {17});
    }
    E.salu("s_add_u32 s23, s8, -1", {23});  // n - 1
    const std::string loop = E.newlab(), exit_ = E.newlab();
    // the ring: the first rows of the wave's first group, loaded before the loop
    ring_reg.clear();
    if (!glds)
      for (size_t q = 0; q < std::min<size_t>(prefetch_depth(), rows.size()); q++) ring_reg.push_back(fresh());
    vnext = tiled ? Limb{} : fresh();
    spill_hwm = 0;
    spills = 0;
    if (spill_on) {  // the wave's spill slots: s35 = wave * 256 S, spill_v = s35 + 4 S lane (S patched below)
      spill_v = fresh();
      E.salu("s_mul_i32 s35, s3, __MG_SPILL_BYTES__", {35});
      E.valu("v_mul_u32_u24_e32 " + VL(spill_v) + ", __MG_SPILL_STRIDE_, v1");
      E.valu("v_lshl_add_u32 " + VL(spill_v) + ", " + VL(spill_v) + ", 2, s35", {35});
    }
    if (glds) {  // the wave's LDS slots: s34 = wave * slots * 256, glds_v = s34 + 4 * lane
      glds_v = fresh();
      E.salu("s_mul_i32 s34, s3, " + hexs(glds_slots() * 256u), {34});
      E.valu("v_lshl_add_u32 " + VL(glds_v) + ", v1, 2, s34", {34});
    }
    if (tiled) {  // s31 = last group index, s32 = the grid stride in groups
      E.salu("s_add_u32 s31, s8, 63", {31});
      E.salu("s_lshr_b32 s31, s31, 6", {31});
      E.salu("s_add_u32 s31, s31, -1", {31});
      E.salu("s_lshr_b32 s32, s17, 6", {32});
    }
    if (!solo) {
      E.salu("s_cmp_lt_u32 s16, s8");
      E.ctl("s_cbranch_scc0 " + exit_);
    }
    E.valu("v_add_u32_e32 v3, s16, v1", {16});
    if (tiled) {
      E.valu("v_lshlrev_b32_e32 v2, 2, v1");  // lane * 4 inside the group's 256-byte row
      E.salu("s_lshr_b32 s30, s16, 6", {30});
      if (solo) E.salu("s_min_u32 s30, s30, s31", {30});  // a block past n reads the last group
      block_base(26, 30);
      page_at[0] = page_at[1] = -1;
    } else {
      E.valu("v_min_u32_e32 v2, s23, v3", {23});
      E.valu("v_lshlrev_b32_e32 v2, 2, v2");
    }
    for (size_t q = 0; q < ring_reg.size(); q++) load_row(ring_reg[q], rows[q], 26, "v2", " (first group)");
    if (glds)
      for (size_t q = 0; q < gdepth; q++) glds_issue(q);  // the first group's first rows
    if (!solo) {
      E.label(loop);
      E.salu("s_cmp_lt_u32 s16, s8");
      E.ctl("s_cbranch_scc0 " + exit_);
    }
    // i = s16 + lane; v3 = i (store offset), v2 = 4 * min(i, n - 1) (load offset: lanes past n reread
    // the last candidate and store nothing); s[24:25] = lanes with i < n; vnext: the same for i + stride
    // (tiled: v2 = 4 * lane, the blocks of this group and the next in s[26:27] / s[28:29]; the last
    // block is whole in memory, so lanes past n read its padding)
    E.valu("v_add_u32_e32 v3, s16, v1", {16});
    if (tiled) {
      E.salu("s_lshr_b32 s30, s16, 6", {30});
      if (solo) E.salu("s_min_u32 s30, s30, s31", {30});
      block_base(26, 30);
      E.salu("s_add_u32 s33, s30, s32", {33});
      E.salu("s_min_u32 s33, s33, s31", {33});
      block_base(28, 33);
      page_at[0] = page_at[1] = -1;
    } else {
      E.valu("v_min_u32_e32 v2, s23, v3", {23});
      E.valu("v_lshlrev_b32_e32 v2, 2, v2");
      E.valu("v_add_u32_e32 " + VL(vnext) + ", s17, v3", {17});
      E.valu("v_min_u32_e32 " + VL(vnext) + ", s23, " + VL(vnext), {23});
      E.valu("v_lshlrev_b32_e32 " + VL(vnext) + ", 2, " + VL(vnext));
    }
    E.valu("v_cmp_gt_u32_e64 s[24:25], s8, v3", {8}, {24, 25});
    E.valu("v_lshlrev_b32_e32 v8, 2, v3");  // watch-row store offset 4 i
    E.salu("s_mov_b64 s[38:39], -1", {38, 39});
    rows_issued = ring_reg.size();
    rows_used = 0;
    loads = 0;
    for (size_t q = 0; q < ring_reg.size(); q++) row_seq[q] = (long)q - (long)ring_reg.size();
    if (glds) {  // rows 0 .. D-1 came in the previous iteration, its last D VMEM loads
      for (size_t q = 0; q < gdepth; q++) gseq[q] = (long)q - (long)gdepth;
      gl_issued = gdepth;
      staged = 0;
      lgkm_n = 0;
    }
    body("");
    if (rows_used != rows.size()) fail("internal: SoA rows left unread");
    if (glds && (gl_issued != rows.size() + gdepth || staged != rows.size())) fail("internal: LDS row queue");
    for (const Limb& l : ring_reg) drop(l);
    if (!tiled) drop(vnext);
    if (glds) drop(glds_v);
    if (spill_on) drop(spill_v);
    ring_reg.clear();
    for (int r = E.vfirst; r < 256; r++)
      if (E.vref[r]) fail("internal: VGPR v" + std::to_string(r) + " still held after the body");
    // verdict byte of the lanes in range
    E.valu("v_cndmask_b32_e64 v7, 0, 1, s[38:39]", {38, 39});
    E.salu("s_mov_b64 exec, s[24:25]");
    E.mem("global_store_byte v3, v7, s[10:11]");
    E.salu("s_mov_b64 exec, -1");
    if (!solo) {
      E.salu("s_add_u32 s16, s16, s17", {16});
      E.ctl("s_branch " + loop);
    }
    E.label(exit_);
    E.ctl("s_waitcnt vmcnt(0)");  // the last iteration's loads for a group past n
    E.ctl("s_endpgm");
    const int nv = std::max(E.vhigh, kV0), ns = std::max(E.shigh, rp_used ? 102 : 56);
    const int accum = (nv + 3) / 4 * 4;
    o << "  .section .rodata,\"a\",@progbits\n  .p2align 6, 0x0\n  .amdhsa_kernel " << name << "\n"
      << "    .amdhsa_group_segment_fixed_size " << eval_lds_bytes() << "\n    .amdhsa_private_segment_fixed_size 0\n"
      << "    .amdhsa_kernarg_size 36\n"
      << "    .amdhsa_user_sgpr_count 2\n    .amdhsa_user_sgpr_kernarg_segment_ptr 1\n"
      << "    .amdhsa_system_sgpr_workgroup_id_x 1\n    .amdhsa_system_vgpr_workitem_id 0\n"
      << "    .amdhsa_next_free_vgpr " << nv << "\n    .amdhsa_next_free_sgpr " << ns << "\n"
      << "    .amdhsa_accum_offset " << accum << "\n    .amdhsa_reserve_vcc 1\n"
      << "    .amdhsa_float_denorm_mode_32 3\n    .amdhsa_float_denorm_mode_16_64 3\n"
      << "  .end_amdhsa_kernel\n";
    if (solo)  // candidates per workgroup of the loop-free solo kernel (engine: eval launch grid)
      o << "  .globl mgj_meta_eval_cpb\n  .p2align 2\n  .type mgj_meta_eval_cpb,@object\nmgj_meta_eval_cpb:\n"
           "  .long 64\n  .size mgj_meta_eval_cpb, 4\n";
    o << "  .text\n";
    labels = E.nlab;
    meta_vgpr[name] = nv;
    meta_sgpr[name] = ns + 6;
    std::string res = o.str();
    if (spill_on) {
      // the spill slots' wave stride: the ds offsets stay below the LDS-staged rows' slots' end
      const size_t at = res.find("__MG_SPILL_BYTES__");
      if (at != std::string::npos) res.replace(at, 18, hexs(spill_stride() * 256u));
      const size_t st = res.find("__MG_SPILL_STRIDE_");
      if (st != std::string::npos) res.replace(st, 18, hexs(spill_stride()));
    }
    return res;
  }

  // the eval kernel's LDS: four waves' row slots (256 B each) when rows are LDS-staged, and four
  // waves' spill slots
  uint32_t eval_lds_bytes() const {
    return (glds ? 4u * glds_slots() * 256u : 0u) + (spill_on ? (solo ? 1u : 4u) * spill_stride() * 256u : 0u);
  }

  int labels = 0;  // label numbers continue across the kernels of one module
  std::string kernel(const std::string& name) {
    E = Emitter();
    E.nlab = labels;
    E.vsoft = vsoft;
    census.clear();
    E.vfirst = kV0 + (int)pool.size();
    E.vhigh = E.vfirst;
    val.assign(P.vwidth.size(), Val{});
    cval.clear();
    auto& o = E.o;
    o << "  .text\n  .globl " << name << "\n  .p2align 8\n  .type " << name << ",@function\n" << name << ":\n";
    // kernel arguments: search (gconsts, start, count, sk, sg, hit, flags, nblk);
    //                   gen    (gconsts, start, count, sk, sg, verdict_out, nblk)
    E.ctl("s_load_dwordx2 s[4:5], s[0:1], 0x0");
    E.ctl("s_load_dwordx8 s[8:15], s[0:1], 0x8");
    if (gen_kernel) {
      E.ctl("s_load_dwordx2 s[16:17], s[0:1], 0x28");
      E.ctl("s_load_dword s19, s[0:1], 0x30");
    } else {
      E.ctl("s_load_dwordx4 s[16:19], s[0:1], 0x28");
    }
    E.valu("v_and_b32_e32 v1, 63, v0");
    E.valu("v_mov_b32_e32 v6, 0");
    E.valu("v_readfirstlane_b32 s3, v0", {}, {3});
    E.salu("s_lshr_b32 s3, s3, 6", {3});
    E.ctl("s_waitcnt lgkmcnt(0)");
    emit_lds_prologue();
    if (gen_kernel) E.salu("s_mov_b32 s18, 0", {18});
    E.salu("s_and_b32 s29, s18, 1", {29});
    // s[42:43] = early ? 0 : ~0 (the early-exit test of every ASSERT)
    E.salu("s_cmp_eq_u32 s29, 0");
    E.salu("s_cselect_b64 s[42:43], -1, 0", {42, 43});
    E.salu("s_and_b32 s20, s8, 0xffffffc0", {20});
    E.salu("s_mov_b32 s21, s9", {21});
    E.salu("s_add_u32 s22, s8, s10", {22});
    E.salu("s_addc_u32 s23, s9, s11", {23});
    E.salu("s_sub_u32 s24, s22, s20", {24});
    E.salu("s_subb_u32 s25, s23, s21", {25});
    E.salu("s_add_u32 s24, s24, 63", {24});
    E.salu("s_addc_u32 s25, s25, 0", {25});
    E.salu("s_lshr_b64 s[24:25], s[24:25], 6", {24, 25});
    E.salu("s_lshl_b32 s26, s2, 2", {26});
    E.salu("s_add_u32 s26, s26, s3", {26});
    E.salu("s_mov_b32 s27, 0", {27});
    E.salu("s_lshl_b32 s28, s19, 2", {28});
    E.salu("s_mov_b64 s[30:31], -1", {30, 31});
    E.salu("s_mov_b64 s[32:33], 0", {32, 33});
    for (const auto& kv : pool) E.valu("v_mov_b32_e32 " + V((uint32_t)kv.second) + ", " + imm(kv.first));
    // the lane half of the lane key: fmix64(lane ^ sk)
    E.valu("v_xor_b32_e32 v2, s12, v1", {12});
    E.valu("v_mov_b32_e32 v3, s13", {13});
    vfmix(2, 3);
    // the call's partial groups, by base (count and sk are dead from here): s[10:11] = the first group's
    // base when start is not group-aligned, s[12:13] = the last group's when end is not, else ~0 — a
    // group is partial iff its base equals one of them (two 64-bit compares at its end instead of nine
    // SALU of bounds arithmetic per group)
    E.salu("s_and_b32 s12, s22, 0xffffffc0", {12});
    E.salu("s_mov_b32 s13, s23", {13});
    E.salu("s_and_b32 s40, s22, 63", {40});
    E.salu("s_cmp_lg_u32 s40, 0");
    E.salu("s_cselect_b64 s[12:13], s[12:13], -1", {12, 13});
    E.salu("s_and_b32 s40, s8, 63", {40});
    E.salu("s_cmp_lg_u32 s40, 0");
    E.salu("s_cselect_b64 s[10:11], s[20:21], -1", {10, 11});
    E.salu("s_movk_i32 s7, 0x40", {7});  // the group-key table is due at the first group
    const std::string loop = E.newlab(), exit_ = E.newlab(), next = E.newlab(), cont = E.newlab();
    E.label(loop);
    // g < ngroups ?
    E.salu("s_sub_u32 s40, s26, s24", {40});
    E.salu("s_subb_u32 s40, s27, s25", {40});
    E.ctl("s_cbranch_scc0 " + exit_);
    E.salu("s_lshl_b64 s[34:35], s[26:27], 6", {34, 35});
    E.salu("s_add_u32 s34, s34, s20", {34});
    E.salu("s_addc_u32 s35, s35, s21", {35});
    if (!gen_kernel) {
      // stop once the group lies at or above the current first hit
      const std::string noearly = E.newlab();
      E.salu("s_cmp_eq_u32 s29, 0");
      E.ctl("s_cbranch_scc1 " + noearly);
      // agent scope, or system scope (sc0 sc1) when peers on other GPUs lower the word (flags bit 1,
      // MG_SEARCH_SYSTEM_SCOPE: the engine sets it when the device mask spans physical GPUs)
      {
        const std::string sys = E.newlab(), got = E.newlab();
        E.salu("s_and_b32 s40, s18, 2", {40});
        E.ctl("s_cbranch_scc1 " + sys);
        E.mem("global_load_dwordx2 v[8:9], v6, s[16:17] sc1", {16, 17});
        E.ctl("s_branch " + got);
        E.label(sys);
        E.mem("global_load_dwordx2 v[8:9], v6, s[16:17] sc0 sc1", {16, 17});
        E.label(got);
      }
      E.ctl("s_waitcnt vmcnt(0)");
      E.valu("v_readfirstlane_b32 s40, v8", {}, {40});
      E.valu("v_readfirstlane_b32 s41, v9", {}, {41});
      E.salu("s_sub_u32 s40, s34, s40", {40});
      E.salu("s_subb_u32 s40, s35, s41", {40});
      E.ctl("s_cbranch_scc0 " + exit_);
      E.label(noearly);
    }
    // G = fmix64((gbase >> 6) ^ sg), gbase >> 6 = (a0 >> 6) + g.  Every 64 groups the wave computes the
    // keys of its next 64 on the VALU (lane l: group g + l * gstride) into v10/v11, and each group reads
    // its own with two v_readlane: 18 SALU per group (fmix64 on the scalar unit, 8 of them multiplies)
    // become 2 VALU + ~0.4 amortised
    if (salu_group_key()) {
      E.salu("s_lshr_b64 s[36:37], s[34:35], 6", {36, 37});
      E.salu("s_xor_b64 s[36:37], s[36:37], s[14:15]", {36, 37});
      sfmix(36);
    } else {
      const std::string have = E.newlab();
      E.salu("s_cmp_lt_u32 s7, 64");
      E.ctl("s_cbranch_scc1 " + have);
      E.valu("v_mul_u32_u24_e32 v10, s28, v1", {28});
      E.valu("v_lshrrev_b64 v[8:9], 6, s[20:21]", {20, 21});
      E.valu("v_add_co_u32_e32 v10, vcc, s26, v10", {26}, {kVCC, kVCC + 1});
      E.valu("v_mov_b32_e32 v11, s27", {27});
      E.valu("v_addc_co_u32_e32 v11, vcc, 0, v11, vcc", {kVCC, kVCC + 1}, {kVCC, kVCC + 1});
      E.valu("v_add_co_u32_e32 v10, vcc, v8, v10", {}, {kVCC, kVCC + 1});
      E.valu("v_addc_co_u32_e32 v11, vcc, v9, v11, vcc", {kVCC, kVCC + 1}, {kVCC, kVCC + 1});
      E.valu("v_xor_b32_e32 v10, s14, v10", {14});
      E.valu("v_xor_b32_e32 v11, s15, v11", {15});
      vfmix(10, 11);
      E.salu("s_mov_b32 s7, 0", {7});
      E.label(have);
      E.valu("v_readlane_b32 s36, v10, s7", {7}, {36});
      E.valu("v_readlane_b32 s37, v11, s7", {7}, {37});
      E.salu("s_add_u32 s7, s7, 1", {7});
    }
    E.valu("v_xor_b32_e32 v4, s36, v2", {36});
    if (!no_kfold())  // v4 ^= v4 >> 16 (grnd)
      E.valu("v_xor_b32_sdwa v4, v4, v4 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1");
    E.valu("v_xor_b32_e32 v5, s37, v3", {37});
    E.salu("s_mov_b64 s[38:39], -1", {38, 39});
    {  // MYTHGPU_JIT_ASM_DIAG_PAD=S,V: S scalar and V vector no-op moves per group (issue-sensitivity
       // timing builds; results unchanged)
      // ,B: B taken branches to the next instruction
      static const std::array<int, 3> pad = [] {
        const char* g = getenv("MYTHGPU_JIT_ASM_DIAG_PAD");
        int a = 0, b = 0, c = 0;
        if (g) sscanf(g, "%d,%d,%d", &a, &b, &c);
        return std::array<int, 3>{std::max(0, std::min(a, 200)), std::max(0, std::min(b, 200)), std::max(0, std::min(c, 200))};
      }();
      for (int q = 0; q < pad[0]; q++) E.salu("s_mov_b32 s40, s40", {40});
      for (int q = 0; q < pad[1]; q++) E.valu("v_mov_b32_e32 v7, 0");
      for (int q = 0; q < pad[2]; q++) {
        const std::string l = E.newlab();
        E.ctl("s_branch " + l);
        E.label(l);
      }
    }
    body(next);
    for (int r = E.vfirst; r < 256; r++)
      if (E.vref[r]) fail("internal: VGPR v" + std::to_string(r) + " still held after the body");
    E.label(next);
    // m = verdict, restricted to [start, end) in a partial group: in place in s[38:39] (search kernels:
    // dead after the group), a copy in s[40:41] (the gen kernel stores the verdict as well)
    const std::string M = gen_kernel ? "s[40:41]" : "s[38:39]";
    const int m0 = gen_kernel ? 40 : 38;
    if (gen_kernel) E.salu("s_mov_b64 s[40:41], s[38:39]", {40, 41});
    {
      const std::string fullg = E.newlab(), part = E.newlab();
      E.salu("s_cmp_eq_u64 s[34:35], s[10:11]");
      E.ctl("s_cbranch_scc1 " + part);
      E.salu("s_cmp_lg_u64 s[34:35], s[12:13]");
      E.ctl("s_cbranch_scc1 " + fullg);
      E.label(part);
      E.valu("v_add_co_u32_e32 v8, vcc, s34, v1", {34}, {kVCC, kVCC + 1});
      E.valu("v_mov_b32_e32 v9, s35", {35});
      E.valu("v_addc_co_u32_e32 v9, vcc, 0, v9, vcc", {kVCC, kVCC + 1}, {kVCC, kVCC + 1});
      E.valu("v_cmp_le_u64_e64 s[44:45], s[8:9], v[8:9]", {8, 9}, {44, 45});
      E.valu("v_cmp_gt_u64_e64 s[46:47], s[22:23], v[8:9]", {22, 23}, {46, 47});
      E.salu("s_and_b64 " + M + ", " + M + ", s[44:45]", {m0, m0 + 1});
      E.salu("s_and_b64 " + M + ", " + M + ", s[46:47]", {m0, m0 + 1});
      E.label(fullg);
    }
    if (gen_kernel) {
      // verdict bytes of the lanes in range: verdict_out[gbase + lane - start]
      E.salu("s_mov_b64 s[44:45], s[38:39]", {44, 45});
      // lanes in range: the partial-group mask built above when not full (s[40:41] = verdict & range)
      // recompute the range alone into exec
      E.valu("v_add_co_u32_e32 v8, vcc, s34, v1", {34}, {kVCC, kVCC + 1});
      E.valu("v_mov_b32_e32 v9, s35", {35});
      E.valu("v_addc_co_u32_e32 v9, vcc, 0, v9, vcc", {kVCC, kVCC + 1}, {kVCC, kVCC + 1});
      E.valu("v_cmp_le_u64_e64 s[46:47], s[8:9], v[8:9]", {8, 9}, {46, 47});
      E.valu("v_cmp_gt_u64_e64 s[48:49], s[22:23], v[8:9]", {22, 23}, {48, 49});
      E.salu("s_and_b64 s[46:47], s[46:47], s[48:49]", {46, 47});
      E.valu("v_cndmask_b32_e64 v7, 0, 1, s[44:45]", {44, 45});
      E.salu("s_sub_u32 s50, s34, s8", {50});
      E.salu("s_subb_u32 s51, s35, s9", {51});
      E.salu("s_add_u32 s50, s50, s16", {50});
      E.salu("s_addc_u32 s51, s51, s17", {51});
      E.valu("v_add_co_u32_e32 v8, vcc, s50, v1", {50}, {kVCC, kVCC + 1});
      E.valu("v_mov_b32_e32 v9, s51", {51});
      E.valu("v_addc_co_u32_e32 v9, vcc, 0, v9, vcc", {kVCC, kVCC + 1}, {kVCC, kVCC + 1});
      E.salu("s_mov_b64 exec, s[46:47]");
      E.mem("global_store_byte v[8:9], v7, off");
      E.salu("s_mov_b64 exec, -1");
    } else {
      // a wave sweeps its groups in increasing index order, so its first group with a hit holds its
      // best: later groups only count (bcnt) — no first-lane search and no 64-bit compare with the best
      E.salu("s_bcnt1_i32_b64 s45, s[38:39]", {45});  // SCC: any hit
      E.ctl("s_cbranch_scc0 " + cont);
      E.salu("s_add_u32 s32, s32, s45", {32});
      E.salu("s_addc_u32 s33, s33, 0", {33});
      E.salu("s_cmp_lg_u64 s[30:31], -1");
      E.ctl("s_cbranch_scc1 " + cont);
      E.salu("s_ff1_i32_b64 s44, s[38:39]", {44});
      E.salu("s_add_u32 s46, s34, s44", {46});
      E.salu("s_addc_u32 s47, s35, 0", {47});
      E.salu("s_mov_b64 s[30:31], s[46:47]", {30, 31});
      E.salu("s_cmp_eq_u32 s29, 0");
      E.ctl("s_cbranch_scc1 " + cont);
      E.salu("s_mov_b64 exec, 1");
      E.valu("v_mov_b32_e32 v8, s46", {46});
      E.valu("v_mov_b32_e32 v9, s47", {47});
      E.mem("global_atomic_umin_x2 v6, v[8:9], s[16:17]", {16, 17});
      // ... and to the devices whose slices lie above this one's: the peer line after the hit
      // buffer (engine.hip kPeerWord: [272] count, [273 + k] their hit words)
      {
        const std::string ploop = E.newlab(), pdone = E.newlab();
        E.mem("global_load_dwordx2 v[8:9], v6, s[16:17] offset:2176", {16, 17});
        E.ctl("s_waitcnt vmcnt(0)");
        E.valu("v_readfirstlane_b32 s48, v8", {}, {48});
        E.salu("s_min_u32 s48, s48, 15", {48});
        E.salu("s_cmp_eq_u32 s48, 0");
        E.ctl("s_cbranch_scc1 " + pdone);
        E.salu("s_mov_b32 s49, 0", {49});
        E.label(ploop);
        E.salu("s_lshl_b32 s52, s49, 3", {52});
        E.salu("s_add_u32 s52, s52, 0x888", {52});  // 2,184 B: the first peer pointer
        E.valu("v_mov_b32_e32 v7, s52", {52});
        E.mem("global_load_dwordx2 v[8:9], v7, s[16:17]", {16, 17});
        E.ctl("s_waitcnt vmcnt(0)");
        E.valu("v_readfirstlane_b32 s50, v8", {}, {50});
        E.valu("v_readfirstlane_b32 s51, v9", {}, {51});
        E.valu("v_mov_b32_e32 v8, s46", {46});
        E.valu("v_mov_b32_e32 v9, s47", {47});
        E.mem("global_atomic_umin_x2 v6, v[8:9], s[50:51] sc1", {50, 51});  // system scope: a peer GPU's word
        E.salu("s_add_u32 s49, s49, 1", {49});
        E.salu("s_cmp_lt_u32 s49, s48");
        E.ctl("s_cbranch_scc1 " + ploop);
        E.label(pdone);
      }
      E.salu("s_mov_b64 exec, -1");
    }
    E.label(cont);
    E.salu("s_add_u32 s26, s26, s28", {26});
    E.salu("s_addc_u32 s27, s27, 0", {27});
    E.ctl("s_branch " + loop);
    E.label(exit_);
    if (!gen_kernel) {
      const std::string nobest = E.newlab(), end = E.newlab();
      E.salu("s_cmp_eq_u64 s[30:31], -1");
      E.ctl("s_cbranch_scc1 " + nobest);
      if (exit_skip()) {
        // every wave's atomicMin on the one hit word serialises at the L2 (C3: most waves hit, 65,536
        // waves at 64 blocks per CU): read the word first and skip the atomic when this wave's best
        // cannot lower it (a stale read is larger than the word, never smaller: at worst one atomic
        // too many)
        E.salu("s_mov_b64 exec, 1");
        E.mem("global_load_dwordx2 v[8:9], v6, s[16:17]", {16, 17});
        E.ctl("s_waitcnt vmcnt(0)");
        E.valu("v_readfirstlane_b32 s46, v8", {}, {46});
        E.valu("v_readfirstlane_b32 s47, v9", {}, {47});
        E.salu("s_mov_b64 exec, -1");
        E.salu("s_sub_u32 s44, s30, s46", {44});
        E.salu("s_subb_u32 s44, s31, s47", {44});  // SCC: best < word
        E.ctl("s_cbranch_scc0 " + nobest);
      }
      E.salu("s_mov_b64 exec, 1");
      E.valu("v_mov_b32_e32 v8, s30", {30});
      E.valu("v_mov_b32_e32 v9, s31", {31});
      E.mem("global_atomic_umin_x2 v6, v[8:9], s[16:17]", {16, 17});
      E.salu("s_mov_b64 exec, -1");
      E.label(nobest);
      E.salu("s_cmp_eq_u64 s[32:33], 0");
      E.ctl("s_cbranch_scc1 " + end);
      // the wave's count goes to its block's stripe (engine.hip kHitStripes: 16 x 128 B after the hit)
      E.salu("s_and_b32 s40, s2, 15", {40});
      E.salu("s_add_u32 s40, s40, 1", {40});
      E.salu("s_lshl_b32 s40, s40, 7", {40});
      E.salu("s_add_u32 s44, s16, s40", {44});
      E.salu("s_addc_u32 s45, s17, 0", {45});
      E.salu("s_mov_b64 exec, 1");
      E.valu("v_mov_b32_e32 v8, s32", {32});
      E.valu("v_mov_b32_e32 v9, s33", {33});
      E.mem("global_atomic_add_x2 v6, v[8:9], s[44:45]", {44, 45});
      E.label(end);
    }
    E.ctl("s_endpgm");
    // descriptor (MYTHGPU_JIT_ASM_DIAG_VGPRS=N: at least N VGPRs reserved — fewer waves per SIMD, for
    // occupancy-sensitivity timing builds)
    static const int diag_vgprs = [] {
      const char* g = getenv("MYTHGPU_JIT_ASM_DIAG_VGPRS");
      return g ? std::max(0, std::min(256, atoi(g))) : 0;
    }();
    const int nv = std::max({E.vhigh, kV0, diag_vgprs}), ns = std::max(E.shigh, 56);
    const int accum = (nv + 3) / 4 * 4;
    o << "  .section .rodata,\"a\",@progbits\n  .p2align 6, 0x0\n  .amdhsa_kernel " << name << "\n"
      << "    .amdhsa_group_segment_fixed_size " << lds_words * 4 << "\n    .amdhsa_private_segment_fixed_size 0\n"
      << "    .amdhsa_kernarg_size " << (gen_kernel ? 52 : 56) << "\n"
      << "    .amdhsa_user_sgpr_count 2\n    .amdhsa_user_sgpr_kernarg_segment_ptr 1\n"
      << "    .amdhsa_system_sgpr_workgroup_id_x 1\n    .amdhsa_system_vgpr_workitem_id 0\n"
      << "    .amdhsa_next_free_vgpr " << nv << "\n    .amdhsa_next_free_sgpr " << ns << "\n"
      << "    .amdhsa_accum_offset " << accum << "\n    .amdhsa_reserve_vcc 1\n"
      << "    .amdhsa_float_denorm_mode_32 3\n    .amdhsa_float_denorm_mode_16_64 3\n"
      << "  .end_amdhsa_kernel\n  .text\n";
    labels = E.nlab;
    meta_lds = lds_words * 4;
    meta_vgpr[name] = nv;
    meta_sgpr[name] = ns + 6;
    return o.str();
  }
  std::map<std::string, int> meta_vgpr, meta_sgpr;
  uint32_t meta_lds = 0;
};

std::string metadata(const std::map<std::string, int>& vg, const std::map<std::string, int>& sg, bool with_gen,
                     uint32_t lds_bytes) {
  std::ostringstream o;
  auto arg = [&](uint32_t off, uint32_t size, const char* kind, bool global) {
    o << "      - .offset: " << off << "\n        .size: " << size << "\n        .value_kind: " << kind << "\n";
    if (global) o << "        .address_space: global\n";
  };
  o << "  .amdgpu_metadata\n---\namdhsa.kernels:\n";
  for (const char* name : {"mgj_search", "mgj_gen"}) {
    const bool gen = std::strcmp(name, "mgj_gen") == 0;
    if (gen && !with_gen) continue;
    o << "  - .args:\n";
    arg(0, 8, "global_buffer", true);
    for (uint32_t k = 0; k < 4; k++) arg(8 + 8 * k, 8, "by_value", false);
    arg(40, 8, "global_buffer", true);
    if (gen) {
      arg(48, 4, "by_value", false);
    } else {
      arg(48, 4, "by_value", false);
      arg(52, 4, "by_value", false);
    }
    o << "    .group_segment_fixed_size: " << lds_bytes << "\n    .kernarg_segment_align: 8\n"
      << "    .kernarg_segment_size: " << (gen ? 52 : 56) << "\n    .max_flat_workgroup_size: 256\n"
      << "    .name: " << name << "\n    .private_segment_fixed_size: 0\n"
      << "    .sgpr_count: " << sg.at(name) << "\n    .sgpr_spill_count: 0\n"
      << "    .symbol: " << name << ".kd\n    .uniform_work_group_size: 1\n    .uses_dynamic_stack: false\n"
      << "    .vgpr_count: " << vg.at(name) << "\n    .vgpr_spill_count: 0\n    .wavefront_size: 64\n"
      << "    .agpr_count: 0\n";
  }
  o << "amdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n  .end_amdgpu_metadata\n";
  return o.str();
}

}  // namespace

std::string metadata_eval(int vg, int sg, uint32_t lds) {
  std::ostringstream o;
  auto arg = [&](uint32_t off, uint32_t size, const char* kind, bool global) {
    o << "      - .offset: " << off << "\n        .size: " << size << "\n        .value_kind: " << kind << "\n";
    if (global) o << "        .address_space: global\n";
  };
  o << "  .amdgpu_metadata\n---\namdhsa.kernels:\n  - .args:\n";
  arg(0, 8, "global_buffer", true);
  arg(8, 8, "by_value", false);
  arg(16, 8, "global_buffer", true);
  arg(24, 8, "global_buffer", true);
  arg(32, 4, "by_value", false);
  o << "    .group_segment_fixed_size: " << lds << "\n    .kernarg_segment_align: 8\n    .kernarg_segment_size: 36\n"
    << "    .max_flat_workgroup_size: 256\n    .name: mgj_eval\n    .private_segment_fixed_size: 0\n"
    << "    .sgpr_count: " << sg << "\n    .sgpr_spill_count: 0\n    .symbol: mgj_eval.kd\n"
    << "    .uniform_work_group_size: 1\n    .uses_dynamic_stack: false\n    .vgpr_count: " << vg
    << "\n    .vgpr_spill_count: 0\n    .wavefront_size: 64\n    .agpr_count: 0\n"
    << "amdhsa.target: amdgcn-amd-amdhsa--gfx950\namdhsa.version:\n  - 1\n  - 2\n...\n  .end_amdgpu_metadata\n";
  return o.str();
}

// SALU : VALU lines of a search kernel's first pass (VALU group key, no caches) below which the group
// key stays on the scalar unit (whole kernel: C2 0.24, C5 0.16: scalar; C1 0.26, etherstore 0.27, C4 0.32,
// C3 0.41: the VALU table)
constexpr double kSgkeyRatio = 0.25;

// the most VGPRs a kernel of `v` VGPRs may use and keep its waves per SIMD (512 per lane, in
// granules of 8), and never below 96 (5 waves)
static int occupancy_step(int v) {
  // MYTHGPU_JIT_ASM_VMIN=N: the floor instead of 96 (diagnostic)
  static const int floor_v = [] {
    const char* g = getenv("MYTHGPU_JIT_ASM_VMIN");
    return g ? std::max(24, std::min(256, atoi(g))) : 96;
  }();
  const int waves = std::max(1, std::min(8, 512 / ((std::max(v, 1) + 7) / 8 * 8)));
  return std::max(floor_v, std::min(256, 512 / waves / 8 * 8));
}

int jit_asm_source(const Lowered& P, const std::vector<GenSpec>& specs, const std::vector<uint32_t>& gconsts,
                   uint32_t kernels, std::string& out, std::string& err) {
  try {
    Gen g(P, specs, gconsts);
    std::ostringstream o;
    o << kAsmMarker << "\n  .amdgcn_target \"amdgcn-amd-amdhsa--gfx950\"\n  .amdhsa_code_object_version 6\n";
    if (kernels & JIT_EVAL) try {  // the eval kernel alone (no generator)
      // MYTHGPU_JIT_ASM_SPILL_TEST=N (tests): straight to the spilling kernel with only N VGPRs
      if (const char* st = getenv("MYTHGPU_JIT_ASM_SPILL_TEST")) throw AsmFail{"out of VGPRs (spill test " + std::string(st) + ")"};
      g.eval_kernel = true;
      g.tiled = (kernels & JIT_EVAL_TILED) || getenv("MYTHGPU_JIT_ASM_TILED");
      g.analyse();
      // The HBM stream is latency-bound (rows in flight per wave x waves per SIMD): the row queue gets
      // the registers the kernel's occupancy step leaves (C2: 44 rows at 4 waves per SIMD; C4: ~40 at 2).
      // MYTHGPU_JIT_ASM_PREFETCH fixes the depth instead.
      g.depth = Gen::prefetch_env() ? Gen::prefetch_env() : 8u;
      // the cache-free kernel's VGPRs set the occupancy step; the cached kernels stay within it
      g.caches = false;
      std::string ks;
      int nv;
      try {
        ks = g.kernel_eval("mgj_eval");
        nv = g.meta_vgpr["mgj_eval"];
      } catch (const AsmFail&) {  // as for the search kernel: no soft limit
        nv = 256;
      }
      const int waves = std::max(1, std::min(8, 512 / ((nv + 7) / 8 * 8)));
      const int budget = std::min(256, 512 / waves / 8 * 8);
      g.caches = true;
      g.vsoft = budget;
      g.labels = 0;
      ks = g.kernel_eval("mgj_eval");
      if (!Gen::prefetch_env()) {
        for (int d = std::min(60, 8 + budget - nv); d > 8; d -= 4) {
          g.depth = (uint32_t)d;
          g.labels = 0;
          try {
            std::string k2 = g.kernel_eval("mgj_eval");
            if (g.meta_vgpr["mgj_eval"] <= budget) {
              ks = k2;
              break;
            }
          } catch (const AsmFail&) {  // out of VGPRs at this depth: a shallower one
            g.meta_vgpr["mgj_eval"] = 1 << 20;
          }
        }
        if (g.meta_vgpr["mgj_eval"] > budget) {  // none fitted: the depth-8 kernel again
          g.depth = 8;
          g.labels = 0;
          ks = g.kernel_eval("mgj_eval");
        }
      }
      // LDS-staged rows (tiled SoA): the queue depth the LDS leaves at the kernel's occupancy (160 KiB
      // per CU over `waves` four-wave workgroups, 2 D + 1 slots of 256 B per wave), taken when deeper
      // than the register queue just sized.  MYTHGPU_JIT_ASM_GLDS=0 keeps the register queue, =N fixes D
      if (g.tiled && Gen::glds_env()) {
        const std::string vks = ks;
        const uint32_t vdepth = g.depth;
        const int vnv = g.meta_vgpr["mgj_eval"];
        const uint32_t M = (uint32_t)g.rows.size();
        auto depth_for = [&](int nv) {
          if (Gen::glds_fixed()) return std::min<uint32_t>(Gen::glds_fixed(), M);
          const int w = std::max(1, std::min(8, 512 / ((nv + 7) / 8 * 8)));
          const int slots = 160 / w;
          return std::min<uint32_t>({32u, M, (uint32_t)std::max(1, (slots - 1) / 2)});
        };
        g.gdepth = depth_for(vnv);
        bool ok = true;
        try {
          g.labels = 0;
          ks = g.kernel_eval("mgj_eval");
          const uint32_t d2 = depth_for(g.meta_vgpr["mgj_eval"]);
          if (d2 != g.gdepth) {
            g.gdepth = d2;
            g.labels = 0;
            ks = g.kernel_eval("mgj_eval");
          }
        } catch (const AsmFail&) {
          ok = false;
        }
        if (!ok || (!Gen::glds_fixed() && g.gdepth <= vdepth)) {  // the register queue is as deep
          g.gdepth = 0;
          g.depth = vdepth;
          g.glds = false;
          ks = vks;
          g.meta_vgpr["mgj_eval"] = vnv;
        }
      }
      if (!getenv("MYTHGPU_JIT_ASM_NOPOOL")) {
        std::vector<std::pair<uint32_t, uint32_t>> by;
        for (const auto& kv : g.census)
          if (kv.second >= 2) by.push_back({kv.second, kv.first});
        std::sort(by.begin(), by.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
        const int room = std::max(0, 96 - g.meta_vgpr["mgj_eval"]);
        for (size_t i = 0; i < by.size() && (int)i < room; i++) g.pool[by[i].second] = kV0 + (int)i;
        if (!g.pool.empty()) {
          g.labels = 0;
          ks = g.kernel_eval("mgj_eval");
        }
      }
      o << ks << metadata_eval(g.meta_vgpr["mgj_eval"], g.meta_sgpr["mgj_eval"], g.eval_lds_bytes());
      out = o.str();
      return MG_OK;
    } catch (const AsmFail& f) {
      // out of VGPRs at every queue depth: once more with spills to LDS (Gen::spill_one), a depth-8
      // register queue and the caches bounded by all 256 registers.  MYTHGPU_JIT_ASM_NO_SPILL=1: refuse
      const char* ns = getenv("MYTHGPU_JIT_ASM_NO_SPILL");
      if ((ns && ns[0] == '1') || f.why.find("out of VGPRs") == std::string::npos) throw;
      Gen g2(P, specs, gconsts);
      g2.eval_kernel = true;
      g2.tiled = (kernels & JIT_EVAL_TILED) || getenv("MYTHGPU_JIT_ASM_TILED");
      g2.analyse();
      g2.spill_on = true;
      g2.depth = 8;
      g2.gdepth = 0;
      g2.caches = true;
      g2.vsoft = 256;
      if (const char* st = getenv("MYTHGPU_JIT_ASM_SPILL_TEST")) g2.vhard = g2.vsoft = std::max(24, std::min(256, atoi(st)));
      g2.labels = 0;
      std::string ks;
      try {
        ks = g2.kernel_eval("mgj_eval");
      } catch (const AsmFail& f2) {
        // more slots than four waves' LDS holds: one working wave per workgroup (Gen::solo)
        if (f2.why.find("spill slots") == std::string::npos) throw;
        g2.solo = true;
        g2.labels = 0;
        ks = g2.kernel_eval("mgj_eval");
      }
      o << ks << metadata_eval(g2.meta_vgpr["mgj_eval"], g2.meta_sgpr["mgj_eval"], g2.eval_lds_bytes());
      out = o.str();
      return MG_OK;
    }
    g.analyse();
    // pass 1, without the value caches, counts the literals the kernel moves into VGPRs and its VGPRs;
    // pass 2 pools the most used literals and runs the caches within the occupancy step pass 1 reached
    // (at least 96 VGPRs, 5 waves per SIMD)
    g.gen_kernel = false;
    g.caches = false;
    std::string ks;
    int v0;
    try {
      ks = g.kernel("mgj_search");
      v0 = g.meta_vgpr["mgj_search"];
      if (getenv("MYTHGPU_JIT_ASM_VREPORT")) fprintf(stderr, "mythgpu asm: pass-1 VGPRs %d\n", v0);
    } catch (const AsmFail&) {
      // out of VGPRs without the caches (shared XOR limbs relieve pressure): no soft limit then
      v0 = 256;
      g.census.clear();
    }
    g.caches = true;
    g.vsoft = occupancy_step(v0);
    // the group key's unit (Gen::sgkey): the scalar unit unless the first pass's body leans on it
    if (Gen::sgkey_env() >= 0) {
      g.sgkey = Gen::sgkey_env() == 1;
    } else if (!ks.empty()) {
      size_t sa = 0, va = 0;
      std::istringstream in(ks);
      for (std::string ln; std::getline(in, ln);) {
        if (ln.rfind("  v_", 0) == 0) va++;
        else if (ln.rfind("  s_", 0) == 0 && ln.rfind("  s_waitcnt", 0) && ln.rfind("  s_nop", 0) &&
                 ln.rfind("  s_branch", 0) && ln.rfind("  s_cbranch", 0) && ln.rfind("  s_endpgm", 0))
          sa++;
      }
      g.sgkey = va && (double)sa < kSgkeyRatio * (double)va;
    }
    {
      std::vector<std::pair<uint32_t, uint32_t>> by;  // (count, literal)
      // MYTHGPU_JIT_ASM_POOL_MIN=N: pool literals materialised at least N times (default 2)
      static const uint32_t pool_min = [] {
        const char* g = getenv("MYTHGPU_JIT_ASM_POOL_MIN");
        return g ? (uint32_t)std::max(1, atoi(g)) : 2u;
      }();
      if (!getenv("MYTHGPU_JIT_ASM_NOPOOL"))
        for (const auto& kv : g.census)
          if (kv.second >= pool_min) by.push_back({kv.second, kv.first});
      std::sort(by.begin(), by.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
      const int room = std::max(0, std::min(96, g.vsoft) - v0);
      for (size_t i = 0; i < by.size() && (int)i < room; i++) g.pool[by[i].second] = kV0 + (int)i;
      g.labels = 0;
      ks = g.kernel("mgj_search");
    }
    o << ks;
    const bool with_gen = (kernels & JIT_GEN) != 0;
    if (with_gen) {
      g.gen_kernel = true;
      o << g.kernel("mgj_gen");
    }
    o << metadata(g.meta_vgpr, g.meta_sgpr, with_gen, g.meta_lds);
    out = o.str();
    return MG_OK;
  } catch (const AsmFail& f) {
    err = f.why;
    return MG_E_UNSUPPORTED;
  } catch (const std::exception& x) {
    err = std::string("assembly tier: ") + x.what();
    return MG_E_UNSUPPORTED;
  }
}

}  // namespace mg
