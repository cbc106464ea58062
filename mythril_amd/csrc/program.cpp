// Program v1 parser, validator and lowering (host C++).
//
// Lowering does three things the kernels rely on:
//  1. arrays/UFs -> per-lane canonicalising lookups: a Select over
//     Store(...Store(A, i1, v1)..., ik, vk) at index j becomes
//     ite(j==ik, vk, ... ite(j==i1, v1, LOOKUP_A(j)) ...), and LOOKUP_A returns
//     the value of the first earlier site of A whose key equals j, else the
//     site's own coordinate (z3 array/UF semantics under a finite model,
//     mythril/laser/smt/array.py:16-63, function.py:7-25);
//  2. a liveness pass + first-fit allocator over 32-bit words gives every value a
//     slot in the per-lane value file (destinations never alias live operands);
//  3. roots become K_ASSERT right after they are computed, so the verdict is a
//     running AND and a wave can stop once all its lanes failed.
#include "program.hpp"

#include <algorithm>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <tuple>
#include <cstdio>
#include <cstdlib>

namespace mg {

static inline uint32_t L_of(uint32_t w) { return (w + 31) / 32; }

uint64_t op_cost(uint32_t k, uint32_t w, uint32_t wa) {
  // SURVEY.md §8(d) fixed cost table, in 32-bit limb operations.
  const uint64_t L = L_of(w), La = L_of(wa);
  switch (k) {
    case K_ADD: case K_SUB: case K_NEG: case K_AND: case K_OR: case K_XOR: case K_NOT:
    case K_ITE: case K_EXTRACT: case K_CONCAT: case K_ZEXT: case K_SEXT:
      return L;
    case K_EQ: case K_ULT: case K_ULE: case K_SLT: case K_SLE:
      return 2 * La;
    case K_SHL: case K_LSHR: case K_ASHR:
      return 4 * L;
    case K_MUL:
      return L * (L + 1) / 2 + L * (L - 1) / 2 + L * L;
    case K_UMUL_NOOVF:
      return 4 * La * La;
    case K_UDIV: case K_UREM: case K_SDIV: case K_SREM: case K_SMOD:
      return 4 * L * L + 16 * L;
    case K_EXP:
      // 128 x (bits + popcount) with the mean popcount of a w-bit exponent
      return 128ull * (uint64_t)(w + w / 2);
    default:
      return 0;
  }
}

namespace {

struct Node {
  uint32_t op, width, a, b, c, p0, p1, p2;
};

struct ArrInfo {
  bool is_table = false;
  uint32_t table = MG_NONE;     // table index when based on an array variable
  uint32_t default_node = MG_NONE;  // K() default node
  std::vector<std::pair<uint32_t, uint32_t>> stores;  // (index node, value node), oldest first
  uint32_t dom = 0, rng = 0;
};

struct VInstr {
  uint32_t op, wd, dst, a, b, c, p0, p1;
  std::vector<uint32_t> prior;  // LOOKUP: flattened (key vid, val vid) pairs
};

struct Fail {
  int code;
  std::string msg;
};

[[noreturn]] void fail(int code, const std::string& m) { throw Fail{code, m}; }

class Alloc {
 public:
  // best fit (smallest free run that holds n words; lowest address on ties): wide values
  // (512-bit keccak arguments next to 8-bit bytes) fragment a first-fit file badly
  uint32_t alloc(uint32_t n) {
    auto best = free_.end();
    for (auto it = free_.begin(); it != free_.end(); ++it)
      if (it->second >= n && (best == free_.end() || it->second < best->second)) best = it;
    if (best != free_.end()) {
      const uint32_t s = best->first;
      if (best->second == n) {
        free_.erase(best);
      } else {
        const uint32_t ns = best->first + n, nl = best->second - n;
        free_.erase(best);
        free_.emplace(ns, nl);
      }
      return s;
    }
    // extend the file; a free run touching the top is grown instead of skipped
    if (!free_.empty()) {
      auto last = std::prev(free_.end());
      if (last->first + last->second == top_) {
        const uint32_t s = last->first;
        free_.erase(last);
        top_ = s + n;
        return s;
      }
    }
    uint32_t s = top_;
    top_ += n;
    return s;
  }
  void release(uint32_t s, uint32_t n) {
    auto it = free_.emplace(s, n).first;
    // merge with next
    auto nx = std::next(it);
    if (nx != free_.end() && it->first + it->second == nx->first) {
      it->second += nx->second;
      free_.erase(nx);
    }
    if (it != free_.begin()) {
      auto pv = std::prev(it);
      if (pv->first + pv->second == it->first) {
        pv->second += it->second;
        free_.erase(it);
      }
    }
  }
  uint32_t high() const { return top_; }

 private:
  std::map<uint32_t, uint32_t> free_;
  uint32_t top_ = 0;
};

// liveness + first-fit slot allocation of an SSA instruction list: fills out.code/aux
// (slot operands, what the interpreter runs), out.vcode/vaux (value ids, what the JIT
// emits), out.value_words and out.limb_ops
// Interpreter superinstructions (slot code only; the JIT's vcode keeps every instruction): a
// compare whose only use is an ASSERT, directly or through one NOT whose only use is the ASSERT,
// becomes one K_ASSERT_CMP at the compare's place.  The verdict is the same AND of the same Bools;
// only the point where the wave may stop early moves up.  MYTHGPU_INTERP_FUSE=0: off.
// every value id an instruction reads
template <class F>
void for_each_use(const VInstr& c, F&& f) {
  const uint32_t NONE = MG_NONE;
  auto use = [&](uint32_t v) {
    if (v != NONE) f(v);
  };
  if (c.op == K_LOOKUP) {
    use(c.a);
    use(c.p0);
    for (uint32_t v : c.prior) use(v);
  } else if (c.op == K_CONCAT || c.op == K_EXTRACT || c.op == K_ZEXT || c.op == K_SEXT || c.op == K_KECCAK ||
             c.op == K_ASSERT || c.op == K_WATCH || c.op == K_COPY) {
    use(c.a);
    use(c.b);
  } else if (c.op != K_CONST && c.op != K_COORD) {
    use(c.a);
    use(c.b);
    use(c.c);
  }
}

// Lookups read only under the else-side of ITE(EQ(x, y), ...) guards (the compiled kernels' list
// only): LASER's storage reads are ITE chains over the writes' keys, ending in the mapping's own
// lookup, so the lookup tests keys the guards above it have already found unequal.  Along an
// else-chain of single-reader ITEs whose conditions are EQs, a single-reader LOOKUP drops each prior
// whose key test (key, k_q) is one of those pairs — that prior cannot match there — and with no
// prior left it is a COPY of its default.  Exact: the dropped tests are false wherever the value is
// read.  MYTHGPU_ITE_PRUNE=0: off.
std::vector<VInstr> prune_guarded_lookups(const std::vector<VInstr>& code_in, size_t nv, bool* changed) {
  static const bool on = [] {
    const char* g = getenv("MYTHGPU_ITE_PRUNE");
    return !(g && g[0] == '0');
  }();
  *changed = false;
  if (!on) return code_in;
  const uint32_t NONE = MG_NONE;
  std::vector<VInstr> code = code_in;
  auto pair = [](uint32_t a, uint32_t b) { return a < b ? std::make_pair(a, b) : std::make_pair(b, a); };
  for (int round = 0; round < 4; round++) {
    std::vector<uint32_t> uses(nv, 0);
    std::vector<int32_t> defk(nv, -1);
    for (size_t k = 0; k < code.size(); k++) {
      const VInstr& c = code[k];
      if (c.dst != NONE && c.dst < nv) defk[c.dst] = (int32_t)k;
      for_each_use(c, [&](uint32_t x) {
        if (x < nv) uses[x]++;
      });
    }
    auto def = [&](uint32_t v) -> VInstr* { return v < nv && defk[v] >= 0 ? &code[(size_t)defk[v]] : nullptr; };
    bool any = false;
    for (size_t k = code.size(); k-- > 0;) {
      if (code[k].op != K_ITE) continue;
      std::set<std::pair<uint32_t, uint32_t>> ne;  // pairs known unequal on the else side
      const VInstr* ite = &code[k];
      while (true) {
        const VInstr* cd = def(ite->a);
        if (!cd || cd->op != K_EQ) break;
        ne.insert(pair(cd->a, cd->b));
        const uint32_t e = ite->c;
        VInstr* ed = def(e);
        if (!ed || uses[e] != 1) break;
        if (ed->op == K_ITE) {
          ite = ed;
          continue;
        }
        if (ed->op == K_LOOKUP) {
          std::vector<uint32_t> keep;
          for (size_t q = 0; q + 1 < ed->prior.size(); q += 2)
            if (!ne.count(pair(ed->a, ed->prior[q]))) {
              keep.push_back(ed->prior[q]);
              keep.push_back(ed->prior[q + 1]);
            }
          if (keep.size() != ed->prior.size()) {
            any = true;
            if (keep.empty()) {
              *ed = VInstr{K_COPY, ed->wd, ed->dst, ed->p0, NONE, NONE, 0, 0, {}};
            } else {
              ed->prior = std::move(keep);
              ed->c = (uint32_t)(ed->prior.size() / 2);
            }
          }
        }
        break;
      }
    }
    if (!any) break;
    *changed = true;
  }
  return code;
}

// The compare of a lookup's result, pushed into the lookup (the compiled kernels' list only):
//   EQ(LOOKUP(k; (k_q, v_q)...; d), x)  ->  LOOKUP(k; (k_q, EQ(v_q, x))...; EQ(d, x))  of width 1
// (the LOOKUP itself goes when nothing else reads it).  Exact: the lookup selects one of the
// v_q / d, and the compare of the selected value is the selected compare.  LASER's keccak
// bookkeeping asserts this shape once per hashed site (the inverse map's entry for keccak(x) is x:
// the default is x itself, so EQ(d, x) is a literal 1, and the priors' values are keys the program
// already compares).  Kept where it removes work: the width-L compare goes, and the n x L limb
// selects too when the LOOKUP goes; a compare of a
// value with itself is a literal, and a pair the program already compares (an EQ, or a LOOKUP key
// test: LLVM's CSE and the first tier's difference cache share those) is counted free.
// The same for an ITE result (a lookup of one prior), and for the ordered compares (ULT, ULE, SLT,
// SLE) of a lookup or ITE with a literal: CMP(ITE(c, a, b), K) -> ITE(c, CMP(a, K), CMP(b, K)), operand
// order kept — a storage read's bounds check then selects Bools instead of 256-bit words, and its
// literal arms fold.  MYTHGPU_EQ_PUSHDOWN=0: off.
std::vector<VInstr> push_eq_into_lookup(const std::vector<VInstr>& code, std::vector<uint32_t>& vwidth,
                                        std::vector<uint32_t>& consts, bool* changed) {
  static const bool on = [] {
    const char* g = getenv("MYTHGPU_EQ_PUSHDOWN");
    return !(g && g[0] == '0');
  }();
  *changed = false;
  if (!on) return code;
  const uint32_t NONE = MG_NONE;
  const size_t nv = vwidth.size();
  std::vector<uint32_t> uses(nv, 0);
  std::vector<int32_t> defk(nv, -1);
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> eq_of;  // compared pair -> EQ result (NONE: a key test)
  // ordered compares this pass created: (op, a, b) -> result (defined before any later reader: each
  // replacement list is emitted at its compare's place, and the map only grows along the list)
  std::map<std::tuple<uint32_t, uint32_t, uint32_t>, uint32_t> ord_of;
  auto pair = [](uint32_t a, uint32_t b) { return a < b ? std::make_pair(a, b) : std::make_pair(b, a); };
  for (size_t k = 0; k < code.size(); k++) {
    const VInstr& c = code[k];
    if (c.dst != NONE && c.dst < nv) defk[c.dst] = (int32_t)k;
    for_each_use(c, [&](uint32_t x) {
      if (x < nv) uses[x]++;
    });
    if (c.op == K_EQ) eq_of.emplace(pair(c.a, c.b), c.dst);
    if (c.op == K_LOOKUP)
      for (size_t q = 0; q + 1 < c.prior.size(); q += 2) eq_of.emplace(pair(c.a, c.prior[q]), NONE);
  }
  std::vector<char> drop(code.size(), 0);
  std::vector<std::vector<VInstr>> at(code.size());  // replacement of a compare
  auto literal = [&](uint32_t v) { return v < nv && defk[v] >= 0 && code[(size_t)defk[v]].op == K_CONST; };
  for (size_t k = 0; k < code.size(); k++) {
    const VInstr& e = code[k];
    // EQ, and the ordered compares against a literal (LASER's bounds checks of a storage read:
    // ULE(ITE(EQ(key, k1), v1, ... LOOKUP ...), 21)); their operand order is kept
    const bool ordered = e.op == K_ULT || e.op == K_ULE || e.op == K_SLT || e.op == K_SLE;
    if ((e.op != K_EQ && !ordered) || e.dst == NONE) continue;
    if (ordered && !literal(e.a) && !literal(e.b)) continue;
    uint32_t lk = NONE, x = NONE;
    int lside = 0;  // the lookup is operand a (0) or b (1)
    for (int side = 0; side < 2 && lk == NONE; side++) {
      const uint32_t s = side ? e.b : e.a, o = side ? e.a : e.b;
      if (s < nv && defk[s] >= 0 && (code[(size_t)defk[s]].op == K_LOOKUP || code[(size_t)defk[s]].op == K_ITE) &&
          !drop[(size_t)defk[s]]) {
        lk = s;
        x = o;
        lside = side;
      }
    }
    if (lk == NONE) continue;
    const VInstr& L = code[(size_t)defk[lk]];
    // an ITE(c, a, b) is a lookup of one prior: EQ(ITE(c, a, b), x) -> ITE(c, EQ(a, x), EQ(b, x))
    const bool ite = L.op == K_ITE;
    const uint32_t n = ite ? 1u : L.c, W = L.wd, Lw = L_of(W), dflt = ite ? L.c : L.p0;
    std::vector<uint32_t> vals;
    if (ite) vals.push_back(L.b);
    else
      for (uint32_t q = 0; q < n; q++) vals.push_back(L.prior[2 * q + 1]);
    vals.push_back(dflt);
    // a compare of two literals folds in both tiers (the ITE's literal arm against a literal x); an
    // ordered compare is a borrow chain (one instruction per limb), an EQ a XOR and an OR per limb
    const uint64_t per = ordered ? (uint64_t)Lw : 2ull * Lw;
    uint64_t cost_new = n;
    for (uint32_t v : vals)
      if (v != x && !(!ordered && eq_of.count(pair(v, x))) && !(literal(v) && literal(x))) cost_new += per;
    // a lookup read elsewhere too stays: then only the compare goes
    const bool single = uses[lk] == 1;
    const uint64_t cost_old = (single ? (uint64_t)n * Lw : 0ull) + per;
    // where the default is x itself (EQ(d, x) a literal 1) the rewrite is kept even against the cost
    // estimate, which counts every limb as live: the priors' values there are CONCATs with literal
    // tails, whose compares fold (C4 on the O3 kernel: 89.4 -> 97.7 G/s; the first tier -2.7 %,
    // `profiles/r04_eq_pushdown3.jsonl`).  MYTHGPU_EQ_PUSHDOWN=1: the cost estimate only
    static const bool force = [] {
      const char* g = getenv("MYTHGPU_EQ_PUSHDOWN");
      return !(g && g[0] == '1');
    }();
    // Against a literal, a compare goes through selects whose other arms fold (LLVM's compare-of-select
    // folding does the same to the O3 kernels): the compares left to compute along the pushed chains —
    // through ITEs and LOOKUPs, however many readers they have, as each reader is pushed in turn — are
    // counted, and up to six are taken for the wide selects that die once every reader is pushed
    // (C4's storage reads: ITE(EQ(k, k1), 21, ITE(EQ(k, k2), 29, LOOKUP(...))) compared with 13 and 21).
    // the distinct values left to compare (a leaf reached along several chains is compared once)
    std::set<uint32_t> leaves;
    std::function<void(uint32_t, int)> left = [&](uint32_t v, int depth) {
      if (leaves.size() > 6) return;
      if (v == x || (literal(v) && literal(x)) || (!ordered && eq_of.count(pair(v, x)))) return;
      if (depth > 0 && v < nv && defk[v] >= 0 && !drop[(size_t)defk[v]]) {
        const VInstr& D = code[(size_t)defk[v]];
        if (D.op == K_ITE) {
          left(D.b, depth - 1);
          left(D.c, depth - 1);
          return;
        }
        if (D.op == K_LOOKUP) {
          left(D.p0, depth - 1);
          for (uint32_t q = 0; q < D.c; q++) left(D.prior[2 * q + 1], depth - 1);
          return;
        }
      }
      leaves.insert(v);
    };
    if (literal(x))
      for (uint32_t v : vals) left(v, 8);
    if (cost_new >= cost_old && !(force && dflt == x) && !(literal(x) && leaves.size() <= 6)) continue;
    std::vector<VInstr> rep;
    uint32_t one = NONE;
    uint32_t zero = NONE;
    auto eq_id = [&](uint32_t v) -> uint32_t {
      if (v == x) {  // x = x, x <= x: 1; x < x: 0
        const bool t = e.op == K_EQ || e.op == K_ULE || e.op == K_SLE;
        uint32_t& c = t ? one : zero;
        if (c == NONE) {
          c = (uint32_t)vwidth.size();
          vwidth.push_back(1);
          rep.push_back(VInstr{K_CONST, 1, c, NONE, NONE, NONE, (uint32_t)consts.size(), 0, {}});
          consts.push_back(t ? 1u : 0u);
        }
        return c;
      }
      if (ordered) {
        const uint32_t ca = lside ? x : v, cb = lside ? v : x;
        auto it = ord_of.find({e.op, ca, cb});
        if (it != ord_of.end()) return it->second;  // the same compare, pushed along another chain
        const uint32_t id = (uint32_t)vwidth.size();
        vwidth.push_back(1);
        rep.push_back(VInstr{e.op, 1, id, ca, cb, NONE, e.p0, e.p1, {}});
        ord_of[{e.op, ca, cb}] = id;
        return id;
      }
      auto it = eq_of.find(pair(v, x));
      if (it != eq_of.end() && it->second != NONE && defk[it->second] >= 0 && (size_t)defk[it->second] < k)
        return it->second;  // an EQ of the same pair, earlier in the list
      const uint32_t id = (uint32_t)vwidth.size();
      vwidth.push_back(1);
      rep.push_back(VInstr{K_EQ, 1, id, v, x, NONE, e.p0, e.p1, {}});
      eq_of[pair(v, x)] = NONE;  // compared from here on (not reusable as a value: defined here)
      return id;
    };
    if (ite) {
      const uint32_t t = eq_id(vals[0]), f = eq_id(dflt);
      rep.push_back(VInstr{K_ITE, 1, e.dst, L.a, t, f, L.p0, L.p1, {}});
    } else {
      VInstr nl{K_LOOKUP, 1, e.dst, L.a, L.b, n, NONE, 0, {}};
      for (uint32_t q = 0; q < n; q++) {
        nl.prior.push_back(L.prior[2 * q]);
        nl.prior.push_back(eq_id(vals[q]));
      }
      nl.p0 = eq_id(dflt);
      rep.push_back(std::move(nl));
    }
    if (single) drop[(size_t)defk[lk]] = 1;
    drop[k] = 1;
    at[k] = std::move(rep);
    *changed = true;
  }
  if (!*changed) return code;
  std::vector<VInstr> out;
  out.reserve(code.size() + 8);
  for (size_t k = 0; k < code.size(); k++) {
    if (!drop[k]) out.push_back(code[k]);
    for (auto& r : at[k]) out.push_back(std::move(r));
  }
  return out;
}

// K_COORD / K_CONST moved to just before their first use (order among them kept)
// The compiled kernels' list: a Bool NOT whose operand is an ordering compare read only by it becomes
// the complementary compare of the swapped operands — not (a <u b) = b <=u a, not (a <=u b) = b <u a,
// signed alike — defined at the compare's place under the NOT's value id (EQ keeps its NOT).  The first
// tier computes ULE / SLE as the negated borrow, so NOT(ULE) had cost two scalar NOTs.
std::vector<VInstr> fold_not_compares(const std::vector<VInstr>& code, size_t nv, bool* changed) {
  std::vector<uint32_t> uses(nv, 0);
  std::vector<int64_t> def(nv, -1);
  for (size_t k = 0; k < code.size(); k++) {
    for_each_use(code[k], [&](uint32_t v) {
      if (v < nv) uses[v]++;
    });
    if (code[k].dst != MG_NONE && code[k].dst < nv) def[code[k].dst] = (int64_t)k;
  }
  std::vector<VInstr> out = code;
  std::vector<char> drop(code.size(), 0);
  for (size_t k = 0; k < code.size(); k++) {
    const VInstr& n = code[k];
    if (n.op != K_NOT || n.wd != 1 || n.a >= nv || uses[n.a] != 1 || def[n.a] < 0) continue;
    VInstr& c = out[def[n.a]];
    uint32_t op;
    switch (c.op) {
      case K_ULT: op = K_ULE; break;
      case K_ULE: op = K_ULT; break;
      case K_SLT: op = K_SLE; break;
      case K_SLE: op = K_SLT; break;
      default: continue;
    }
    c.op = op;
    std::swap(c.a, c.b);
    c.dst = n.dst;
    drop[k] = 1;
    *changed = true;
  }
  std::vector<VInstr> r;
  r.reserve(out.size());
  for (size_t k = 0; k < out.size(); k++)
    if (!drop[k]) r.push_back(std::move(out[k]));
  return r;
}

std::vector<VInstr> sink_inputs(const std::vector<VInstr>& code, size_t nv) {
  std::vector<int64_t> first(nv, -1);
  for (size_t k = 0; k < code.size(); k++)
    for_each_use(code[k], [&](uint32_t v) {
      if (v < nv && first[v] < 0) first[v] = (int64_t)k;
    });
  std::vector<std::vector<size_t>> before(code.size());
  std::vector<char> moved(code.size(), 0);
  for (size_t k = 0; k < code.size(); k++) {
    const VInstr& c = code[k];
    if ((c.op == K_COORD || c.op == K_CONST) && c.dst < nv && first[c.dst] > (int64_t)k) {
      before[(size_t)first[c.dst]].push_back(k);
      moved[k] = 1;
    }
  }
  std::vector<VInstr> out;
  out.reserve(code.size());
  for (size_t k = 0; k < code.size(); k++) {
    for (size_t m : before[k]) out.push_back(code[m]);
    if (!moved[k]) out.push_back(code[k]);
  }
  return out;
}

std::vector<VInstr> fuse_asserts(const std::vector<VInstr>& code, size_t nv) {
  static const bool on = [] {
    const char* g = getenv("MYTHGPU_INTERP_FUSE");
    return !(g && g[0] == '0');
  }();
  if (!on) return code;
  const uint32_t NONE = MG_NONE;
  std::vector<uint32_t> uses(nv, 0);
  std::vector<int64_t> user(nv, -1);
  auto use = [&](uint32_t v, size_t k) {
    if (v != NONE && v < nv) {
      uses[v]++;
      user[v] = (int64_t)k;
    }
  };
  for (size_t k = 0; k < code.size(); k++) {
    const VInstr& c = code[k];
    if (c.op == K_LOOKUP) {
      use(c.a, k);
      use(c.p0, k);
      for (uint32_t v : c.prior) use(v, k);
    } else if (c.op == K_CONCAT || c.op == K_EXTRACT || c.op == K_ZEXT || c.op == K_SEXT || c.op == K_KECCAK ||
               c.op == K_ASSERT || c.op == K_WATCH || c.op == K_COPY) {
      use(c.a, k);
      use(c.b, k);
    } else if (c.op != K_CONST && c.op != K_COORD) {
      use(c.a, k);
      use(c.b, k);
      use(c.c, k);
    }
  }
  std::vector<char> drop(code.size(), 0);
  std::vector<VInstr> out;
  out.reserve(code.size());
  for (size_t k = 0; k < code.size(); k++) {
    if (drop[k]) continue;
    const VInstr& c = code[k];
    const bool cmp = c.op == K_EQ || c.op == K_ULT || c.op == K_ULE || c.op == K_SLT || c.op == K_SLE;
    if (cmp && c.dst != NONE && c.dst < nv && uses[c.dst] == 1) {
      int64_t u = user[c.dst];
      uint32_t neg = 0;
      int64_t mid = -1;
      if (code[u].op == K_NOT && code[u].wd == 1 && code[u].dst != NONE && code[u].dst < nv &&
          uses[code[u].dst] == 1) {
        mid = u;
        neg = 1;
        u = user[code[u].dst];
      }
      if (code[u].op == K_ASSERT) {
        if (mid >= 0) drop[mid] = 1;
        drop[u] = 1;
        out.push_back(VInstr{K_ASSERT_CMP, 1, NONE, c.a, c.b, NONE, c.op | (neg << 8), c.p1, {}});
        continue;
      }
    }
    out.push_back(c);
  }
  return out;
}

// liveness and best-fit slots of the interpreter's slot code; returns the value file's words.
// code[0, n_hoisted) are K_CONSTs whose slots stay reserved to the end.
uint32_t assign_slots(const std::vector<VInstr>& code, uint32_t n_hoisted, const std::vector<uint32_t>& vwidth,
                      std::vector<Instr>& ocode, std::vector<uint32_t>& oaux) {
  const uint32_t NONE = MG_NONE;
  const size_t nv = vwidth.size();
  std::vector<int64_t> last(nv, -1), def(nv, -1);
  for (size_t k = 0; k < code.size(); k++) {
    const VInstr& c = code[k];
    auto use = [&](uint32_t v) {
      if (v != NONE && v < nv) last[v] = (int64_t)k;
    };
    if (c.op == K_LOOKUP) {
      use(c.a);
      use(c.p0);
      for (uint32_t v : c.prior) use(v);
    } else if (c.op == K_CONCAT || c.op == K_EXTRACT || c.op == K_ZEXT || c.op == K_SEXT ||
               c.op == K_KECCAK || c.op == K_ASSERT || c.op == K_WATCH || c.op == K_COPY) {
      use(c.a);
      use(c.b);
    } else if (c.op != K_CONST && c.op != K_COORD) {
      use(c.a);
      use(c.b);
      use(c.c);
    }
    if (c.dst != NONE && def[c.dst] < 0) def[c.dst] = (int64_t)k;
  }
  for (uint32_t k = 0; k < n_hoisted; k++)
    if (code[k].dst != NONE && code[k].dst < nv) last[code[k].dst] = (int64_t)code.size() - 1;
  std::vector<uint32_t> slot(nv, NONE);
  std::vector<std::vector<uint32_t>> dies(code.size());
  for (size_t v = 0; v < nv; v++) {
    if (def[v] < 0) continue;
    int64_t d = std::max(last[v], def[v]);
    dies[(size_t)d].push_back((uint32_t)v);
  }
  Alloc al;
  uint32_t dbg_high = 0;
  ocode.clear();
  oaux.clear();
  for (size_t k = 0; k < code.size(); k++) {
    VInstr c = code[k];
    if (c.dst != NONE && slot[c.dst] == NONE) slot[c.dst] = al.alloc(L_of(vwidth[c.dst]));
    auto S = [&](uint32_t v) -> uint32_t {
      if (v == NONE) return NONE;
      if (slot[v] == NONE) fail(MG_E_INVALID, "internal: use before definition");
      return slot[v];
    };
    Instr in{c.op, c.wd, c.dst == NONE ? NONE : slot[c.dst], 0, 0, 0, c.p0, c.p1};
    if (c.op == K_LOOKUP) {
      in.a = S(c.a);
      in.b = c.b;
      in.c = c.c;
      in.p0 = S(c.p0);
      in.p1 = (uint32_t)oaux.size();
      for (uint32_t v : c.prior) oaux.push_back(S(v));
    } else if (c.op == K_CONCAT || c.op == K_EXTRACT || c.op == K_ZEXT || c.op == K_SEXT || c.op == K_KECCAK ||
               c.op == K_ASSERT || c.op == K_WATCH || c.op == K_COPY) {
      in.a = S(c.a);
      in.b = S(c.b);
      in.c = NONE;
    } else if (c.op == K_CONST || c.op == K_COORD) {
      in.a = in.b = in.c = NONE;
    } else {
      in.a = S(c.a);
      in.b = S(c.b);
      in.c = S(c.c);
    }
    ocode.push_back(in);
    for (uint32_t v : dies[k]) al.release(slot[v], L_of(vwidth[v]));
    static const bool debug_alloc = getenv("MYTHGPU_DEBUG_ALLOC") != nullptr;
    if (debug_alloc && al.high() > dbg_high) {
      dbg_high = al.high();
      size_t live = 0;
      std::string s;
      for (size_t v = 0; v < nv; v++)
        if (def[v] >= 0 && def[v] <= (int64_t)k && std::max(last[v], def[v]) > (int64_t)k) {
          live += L_of(vwidth[v]);
          s += " " + std::to_string(v) + ":" + std::to_string(vwidth[v]) + "@" + std::to_string(code[def[v]].op) +
               "-" + std::to_string(last[v]);
        }
      fprintf(stderr, "instr %zu high %u live %zu:%s\n", k, al.high(), live, s.c_str());
    }
  }
  return std::max<uint32_t>(al.high(), 1);
}

void allocate(const std::vector<VInstr>& vlist, const std::vector<uint32_t>& vwidth, Lowered& out,
              const std::vector<VInstr>* slot_list = nullptr, bool search_orders = true) {
  const uint32_t NONE = MG_NONE;
  const size_t nv = vwidth.size();
  out.vcode.clear();
  out.vaux.clear();
  // the JIT's SSA list and the cost table: every instruction
  for (const VInstr& c : vlist) {
    Instr vi{c.op, c.wd, c.dst, c.a, c.b, c.c, c.p0, c.p1};
    if (c.op == K_LOOKUP) {
      vi.p1 = (uint32_t)out.vaux.size();
      for (uint32_t v : c.prior) out.vaux.push_back(v);
    }
    out.vcode.push_back(vi);
    uint32_t wa = c.p1;
    if (c.op == K_LOOKUP) {
      out.limb_ops += 3ull * L_of(c.b) * c.c + L_of(c.wd);
    } else if (c.op == K_KECCAK) {
      out.limb_ops += 7500ull * (c.p0 / 136 + 1);
    } else {
      out.limb_ops += op_cost(c.op, c.wd, wa ? wa : c.wd);
    }
  }
  // the interpreter's slot code: superinstructions, then liveness and slots
  // (slot_list: a different program with the same verdicts for the interpreter, e.g. narrowed)
  out.ivcode.clear();
  out.ivaux.clear();
  if (slot_list)
    for (const VInstr& c : *slot_list) {
      Instr vi{c.op, c.wd, c.dst, c.a, c.b, c.c, c.p0, c.p1};
      if (c.op == K_LOOKUP) {
        vi.p1 = (uint32_t)out.ivaux.size();
        for (uint32_t v : c.prior) out.ivaux.push_back(v);
      }
      out.ivcode.push_back(vi);
    }
  const std::vector<VInstr> fused = fuse_asserts(slot_list ? *slot_list : vlist, nv);
  // coordinates (and literals) sunk to just before their first use: a COORD has no inputs (the
  // generator regenerates a COPY's source itself), so its value need not sit in the value file
  // from the top of the program — the file is what limits the interpreter's waves per CU — and a
  // wave that stops at an earlier assert never generates it.  MYTHGPU_INTERP_SINK=0: in place
  static const bool sink_on = [] {
    const char* g = getenv("MYTHGPU_INTERP_SINK");
    return !(g && g[0] == '0');
  }();
  // the smallest value file over {as is, sunk} x {literals in place, hoisted}; ties prefer sunk
  // and hoisted.  Literals do not change from one candidate to the next: with the K_CONSTs first
  // and their slots kept to the end, the interpreter writes them once per thread instead of once
  // per candidate — unless that makes the value file larger (fewer waves per CU cost more than the
  // CONSTs: C2 was 13 % slower with two pinned 256-bit literals).  MYTHGPU_INTERP_HOIST=0: never
  static const bool hoist = [] {
    const char* g = getenv("MYTHGPU_INTERP_HOIST");
    return !(g && g[0] == '0');
  }();
  std::vector<std::vector<VInstr>> orders;
  if (sink_on && search_orders) orders.push_back(sink_inputs(fused, nv));
  orders.push_back(fused);

  bool have = false;
  for (const auto& code : orders) {
    for (int hz = hoist && search_orders ? 1 : 0; hz >= 0; hz--) {
      std::vector<VInstr> h = code;
      uint32_t nh = 0;
      if (hz) {
        std::stable_partition(h.begin(), h.end(), [](const VInstr& c) { return c.op == K_CONST; });
        while (nh < h.size() && h[nh].op == K_CONST) nh++;
        if (!nh) continue;
      }
      std::vector<Instr> hc;
      std::vector<uint32_t> ha;
      const uint32_t words = assign_slots(h, nh, vwidth, hc, ha);
      if (!have || words < out.value_words) {
        out.code.swap(hc);
        out.aux.swap(ha);
        out.value_words = words;
        out.n_hoisted = nh;
        have = true;
      }
    }
  }
  out.vwidth = vwidth;
  static const bool debug_words = getenv("MYTHGPU_DEBUG_ALLOC") != nullptr;
  if (debug_words) fprintf(stderr, "value_words %u n_hoisted %u instrs %zu\n", out.value_words, out.n_hoisted, out.code.size());
}

}  // namespace

int lower_program(const uint8_t* blob, size_t len, Lowered& out, std::string& err) {
  try {
    if (blob == nullptr || len < 64 || (len % 4) != 0) fail(MG_E_INVALID, "program blob too short");
    std::vector<uint32_t> w(len / 4);
    std::memcpy(w.data(), blob, len);
    if (w[0] != MG_MAGIC) fail(MG_E_INVALID, "bad magic");
    if (w[1] != MG_VERSION) fail(MG_E_INVALID, "unsupported program version");
    const uint64_t n_nodes = w[2], n_roots = w[3], n_coords = w[4], n_tables = w[5], n_consts = w[6],
                   n_watch = w[7];
    const uint64_t need = 16 + n_nodes * 8 + n_roots + n_coords * 4 + n_tables * 4 + n_watch + n_consts;
    if (need != w.size()) fail(MG_E_INVALID, "program length does not match header");
    if (n_nodes == 0) fail(MG_E_INVALID, "empty program");
    size_t pos = 16;
    std::vector<Node> nodes(n_nodes);
    for (uint64_t i = 0; i < n_nodes; i++, pos += 8) std::memcpy(&nodes[i], &w[pos], 32);
    std::vector<uint32_t> roots(w.begin() + pos, w.begin() + pos + n_roots);
    pos += n_roots;
    struct C4 { uint32_t width, kind, node, table; };
    std::vector<C4> coords(n_coords);
    for (uint64_t i = 0; i < n_coords; i++, pos += 4) std::memcpy(&coords[i], &w[pos], 16);
    struct T4 { uint32_t kind, kw, vw, z; };
    std::vector<T4> tables(n_tables);
    for (uint64_t i = 0; i < n_tables; i++, pos += 4) std::memcpy(&tables[i], &w[pos], 16);
    std::vector<uint32_t> watch(w.begin() + pos, w.begin() + pos + n_watch);
    pos += n_watch;
    std::vector<uint32_t> consts(w.begin() + pos, w.begin() + pos + n_consts);

    out = Lowered();
    out.n_nodes = (uint32_t)n_nodes;
    out.n_roots = (uint32_t)n_roots;
    out.n_coords = (uint32_t)n_coords;
    out.n_watch = (uint32_t)n_watch;
    out.consts = consts;

    // coordinates
    out.coord_width.resize(n_coords);
    out.coord_row.resize(n_coords);
    out.coord_kind.resize(n_coords);
    out.coord_lazy.assign(n_coords, MG_NONE);
    uint32_t row = 0;
    for (uint64_t c = 0; c < n_coords; c++) {
      if (coords[c].width == 0 || coords[c].width > MG_MAX_WIDTH) fail(MG_E_UNSUPPORTED, "coordinate width");
      if (coords[c].kind > MG_COORD_AUX) fail(MG_E_INVALID, "coordinate kind");
      if (coords[c].node >= n_nodes) fail(MG_E_INVALID, "coordinate node");
      out.coord_width[c] = coords[c].width;
      out.coord_kind[c] = coords[c].kind;
      out.coord_row[c] = row;
      row += L_of(coords[c].width);
    }
    out.coord_words = row;
    for (auto& t : tables) {
      if (t.kind > MG_TABLE_UF || t.kw == 0 || t.vw == 0 || t.kw > MG_MAX_WIDTH || t.vw > MG_MAX_WIDTH)
        fail(MG_E_INVALID, "table descriptor");
    }

    // ---- validate nodes + lower to virtual instructions ---------------
    const uint32_t NONE = MG_NONE;
    std::vector<uint32_t> vid(n_nodes, NONE);
    std::vector<uint32_t> vwidth;  // width per vid
    std::vector<ArrInfo> arr(n_nodes);
    std::vector<char> is_arr(n_nodes, 0);
    std::vector<VInstr> code;
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> table_sites(n_tables);
    std::vector<uint32_t> site_base_vid(n_coords, NONE);
    std::vector<char> root_of(n_nodes, 0), watch_of(n_nodes, 0);
    for (uint32_t r : roots) {
      if (r >= n_nodes) fail(MG_E_INVALID, "root index");
      root_of[r] = 1;
    }
    std::vector<uint32_t> watch_row(n_watch);
    uint32_t wrow = 0;
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> watch_at(n_nodes);  // node -> (watch idx, row)
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> watch_site(n_coords);
    uint32_t max_w = 0;

    std::vector<uint32_t> vconst;  // const-pool offset when the vid is a literal, else NONE
    auto new_vid = [&](uint32_t width) {
      vwidth.push_back(width);
      vconst.push_back(NONE);
      return (uint32_t)(vwidth.size() - 1);
    };
    // two keys that are distinct literals can never select the same table entry:
    // such priors are dropped from a lookup's candidate list at load time
    auto distinct_literals = [&](uint32_t x, uint32_t y) {
      if (vconst[x] == NONE || vconst[y] == NONE || vwidth[x] != vwidth[y]) return false;
      const uint32_t L = L_of(vwidth[x]);
      return std::memcmp(&consts[vconst[x]], &consts[vconst[y]], 4 * L) != 0;
    };
    auto emit = [&](uint32_t op, uint32_t wd, uint32_t dst, uint32_t a = MG_NONE, uint32_t b = MG_NONE, uint32_t c = MG_NONE,
                    uint32_t p0 = 0, uint32_t p1 = 0) {
      VInstr v{op, wd, dst, a, b, c, p0, p1, {}};
      code.push_back(v);
      return code.size() - 1;
    };
    // index of the single set bit of a literal (power of two), else -1
    auto pow2_literal = [&](uint32_t off, uint32_t width) -> int {
      int bit = -1;
      for (uint32_t j = 0; j < L_of(width); j++) {
        const uint32_t x = consts[off + j];
        if (!x) continue;
        if ((x & (x - 1)) || bit >= 0) return -1;
        bit = (int)(32 * j + __builtin_ctz(x));
      }
      return bit;
    };
    // a fresh all-zero literal of the given width (appended to the constant pool)
    auto zero_literal = [&](uint32_t width) -> uint32_t {
      const uint32_t off = (uint32_t)out.consts.size();
      out.consts.insert(out.consts.end(), L_of(width), 0u);
      uint32_t v = new_vid(width);
      emit(K_CONST, width, v, NONE, NONE, NONE, off);
      return v;
    };
    // literals are rematerialised at every use (a scalar-load K_CONST right before
    // the consumer) instead of occupying value-file words from first to last use
    std::vector<uint32_t> node_const(n_nodes, NONE);
    auto val = [&](uint32_t i, uint32_t cur) -> uint32_t {
      if (i >= cur) fail(MG_E_INVALID, "operand does not precede its use");
      if (is_arr[i]) fail(MG_E_INVALID, "array used as a value");
      if (node_const[i] != NONE) {
        uint32_t v = new_vid(nodes[i].width);
        vconst[v] = node_const[i];
        emit(K_CONST, nodes[i].width, v, NONE, NONE, NONE, node_const[i]);
        return v;
      }
      return vid[i];
    };
    uint32_t cur_node = 0;  // operands must precede the node that reads them
    auto wid = [&](uint32_t x) {
      if (x >= cur_node) fail(MG_E_INVALID, "operand does not precede its use");
      return nodes[x].width;
    };

    for (uint32_t i = 0; i < n_nodes; i++) {
      cur_node = i;
      const Node& n = nodes[i];
      const uint32_t W = n.width;
      if (n.op >= MG_OP_COUNT) fail(MG_E_UNSUPPORTED, "unknown operator");
      const bool array_op = n.op == MG_OP_ARR_VAR || n.op == MG_OP_ARR_K || n.op == MG_OP_ARR_STORE;
      if (!array_op) {
        if (W == 0 || W > MG_MAX_WIDTH) fail(MG_E_UNSUPPORTED, "value width");
        max_w = std::max(max_w, W);
      }
      auto need_same = [&](uint32_t a, uint32_t b) {
        if (wid(a) != wid(b)) fail(MG_E_INVALID, "operand width mismatch");
      };
      auto need_le256 = [&](uint32_t width) {
        if (width > 256) fail(MG_E_UNSUPPORTED, "arithmetic wider than 256 bits");
      };
      switch (n.op) {
        case MG_OP_CONST: {
          if ((uint64_t)n.p0 + L_of(W) > n_consts) fail(MG_E_INVALID, "constant out of range");
          node_const[i] = n.p0;  // materialised lazily by val()
          break;
        }
        case MG_OP_VAR: {
          if (n.p0 >= n_coords || (coords[n.p0].kind != MG_COORD_SCALAR && coords[n.p0].kind != MG_COORD_AUX) ||
              coords[n.p0].width != W)
            fail(MG_E_INVALID, "VAR coordinate");
          vid[i] = new_vid(W);
          emit(K_COORD, W, vid[i], NONE, NONE, NONE, n.p0, out.coord_row[n.p0]);
          break;
        }
        case MG_OP_ADD: case MG_OP_SUB: case MG_OP_AND: case MG_OP_OR: case MG_OP_XOR:
        case MG_OP_MUL: case MG_OP_UDIV: case MG_OP_UREM: case MG_OP_SDIV: case MG_OP_SREM:
        case MG_OP_SMOD: case MG_OP_SHL: case MG_OP_LSHR: case MG_OP_ASHR: case MG_OP_EXP: {
          need_same(n.a, n.b);
          if (wid(n.a) != W) fail(MG_E_INVALID, "result width");
          // Strength reduction by a literal power of two (the rewrite z3's simplifier
          // applies too; exact for every operand value):
          //   a udiv 2^k = zext(extract(w-1, k, a)),  a urem 2^k = zext(extract(k-1, 0, a)),
          //   a * 2^k    = extract(w-k-1, 0, a) ++ 0_k
          if ((n.op == MG_OP_UDIV || n.op == MG_OP_UREM || n.op == MG_OP_MUL) && node_const[n.b] != NONE) {
            const int k2 = pow2_literal(node_const[n.b], W);
            if (k2 >= 0 && (uint32_t)k2 < W) {
              const uint32_t k = (uint32_t)k2;
              const uint32_t a = val(n.a, i);
              if (n.op == MG_OP_UDIV) {
                if (k == 0) {
                  vid[i] = a;
                } else {
                  uint32_t t = new_vid(W - k);
                  emit(K_EXTRACT, W - k, t, a, NONE, NONE, k, W);
                  vid[i] = new_vid(W);
                  emit(K_ZEXT, W, vid[i], t, NONE, NONE, 0, W - k);
                }
              } else if (n.op == MG_OP_UREM) {
                if (k == 0) {
                  vid[i] = zero_literal(W);
                } else {
                  uint32_t t = new_vid(k);
                  emit(K_EXTRACT, k, t, a, NONE, NONE, 0, W);
                  vid[i] = new_vid(W);
                  emit(K_ZEXT, W, vid[i], t, NONE, NONE, 0, k);
                }
              } else {  // MUL
                if (k == 0) {
                  vid[i] = a;
                } else {
                  uint32_t t = new_vid(W - k);
                  emit(K_EXTRACT, W - k, t, a, NONE, NONE, 0, W);
                  uint32_t z = zero_literal(k);
                  vid[i] = new_vid(W);
                  emit(K_CONCAT, W, vid[i], t, z, NONE, 0, k);
                }
              }
              break;
            }
          }
          uint32_t a = val(n.a, i), b = val(n.b, i);
          static const uint32_t map[] = {0, 0, K_ADD, K_SUB, K_MUL, K_UDIV, K_UREM, K_SDIV, K_SREM, K_SMOD,
                                         K_AND, K_OR, K_XOR, 0, 0, K_SHL, K_LSHR, K_ASHR};
          uint32_t k = n.op == MG_OP_EXP ? (uint32_t)K_EXP : map[n.op];
          if (k != K_ADD && k != K_SUB && k != K_AND && k != K_OR && k != K_XOR) need_le256(W);
          vid[i] = new_vid(W);
          emit(k, W, vid[i], a, b, NONE, 0, W);
          break;
        }
        case MG_OP_NOT: case MG_OP_NEG: {
          uint32_t a = val(n.a, i);
          if (wid(n.a) != W) fail(MG_E_INVALID, "result width");
          vid[i] = new_vid(W);
          emit(n.op == MG_OP_NOT ? K_NOT : K_NEG, W, vid[i], a, NONE, NONE, 0, W);
          break;
        }
        case MG_OP_CONCAT: {
          uint32_t a = val(n.a, i), b = val(n.b, i);
          if ((uint64_t)wid(n.a) + wid(n.b) != W) fail(MG_E_INVALID, "concat width");
          vid[i] = new_vid(W);
          emit(K_CONCAT, W, vid[i], a, b, NONE, 0, wid(n.b));
          break;
        }
        case MG_OP_EXTRACT: {
          uint32_t a = val(n.a, i);
          if ((uint64_t)n.p0 + W > wid(n.a)) fail(MG_E_INVALID, "extract range");
          vid[i] = new_vid(W);
          emit(K_EXTRACT, W, vid[i], a, NONE, NONE, n.p0, wid(n.a));
          break;
        }
        case MG_OP_ZEXT: case MG_OP_SEXT: {
          uint32_t a = val(n.a, i);
          if (wid(n.a) >= W) fail(MG_E_INVALID, "extend width");
          vid[i] = new_vid(W);
          emit(n.op == MG_OP_ZEXT ? K_ZEXT : K_SEXT, W, vid[i], a, NONE, NONE, 0, wid(n.a));
          break;
        }
        case MG_OP_ITE: {
          uint32_t a = val(n.a, i), b = val(n.b, i), c = val(n.c, i);
          if (wid(n.a) != 1 || wid(n.b) != W || wid(n.c) != W) fail(MG_E_INVALID, "ite widths");
          vid[i] = new_vid(W);
          emit(K_ITE, W, vid[i], a, b, c, 0, W);
          break;
        }
        case MG_OP_EQ: case MG_OP_ULT: case MG_OP_ULE: case MG_OP_SLT: case MG_OP_SLE:
        case MG_OP_UMUL_NOOVF: {
          uint32_t a = val(n.a, i), b = val(n.b, i);
          need_same(n.a, n.b);
          if (W != 1) fail(MG_E_INVALID, "predicate width");
          static const uint32_t map[] = {K_EQ, K_ULT, K_ULE, K_SLT, K_SLE, K_UMUL_NOOVF};
          uint32_t k = map[n.op - MG_OP_EQ];
          if (k == K_UMUL_NOOVF) need_le256(wid(n.a));
          vid[i] = new_vid(1);
          emit(k, 1, vid[i], a, b, NONE, 0, wid(n.a));
          break;
        }
        case MG_OP_ARR_VAR: {
          if (n.p0 >= n_tables || tables[n.p0].kind != MG_TABLE_ARRAY) fail(MG_E_INVALID, "array table");
          is_arr[i] = 1;
          arr[i].is_table = true;
          arr[i].table = n.p0;
          arr[i].dom = tables[n.p0].kw;
          arr[i].rng = tables[n.p0].vw;
          break;
        }
        case MG_OP_ARR_K: {
          if (n.a >= i || is_arr[n.a]) fail(MG_E_INVALID, "K default");
          is_arr[i] = 1;
          arr[i].default_node = n.a;
          arr[i].rng = wid(n.a);
          arr[i].dom = 0;  // any
          break;
        }
        case MG_OP_ARR_STORE: {
          if (n.a >= i || !is_arr[n.a]) fail(MG_E_INVALID, "store base");
          if (n.b >= i || n.c >= i || is_arr[n.b] || is_arr[n.c]) fail(MG_E_INVALID, "store operands");
          is_arr[i] = 1;
          arr[i] = arr[n.a];
          if (arr[i].dom == 0) arr[i].dom = wid(n.b);
          if (wid(n.b) != arr[i].dom || wid(n.c) != arr[i].rng) fail(MG_E_INVALID, "store sorts");
          arr[i].stores.emplace_back(n.b, n.c);
          break;
        }
        case MG_OP_SELECT: {
          if (n.a >= i || !is_arr[n.a]) fail(MG_E_INVALID, "select array");
          const ArrInfo& A = arr[n.a];
          uint32_t key = val(n.b, i);
          if (A.dom && wid(n.b) != A.dom) fail(MG_E_INVALID, "select index width");
          if (A.rng != W) fail(MG_E_INVALID, "select width");
          uint32_t cur;
          if (A.is_table) {
            if (n.p0 >= n_coords || coords[n.p0].kind != MG_COORD_ARRAY_SITE || coords[n.p0].table != A.table ||
                coords[n.p0].width != W)
              fail(MG_E_INVALID, "select site coordinate");
            uint32_t dflt;
            if (n.p1 != NONE) {  // lazy default: a program node (e.g. a byte of an AUX calldata word)
              if (n.p1 >= i || is_arr[n.p1] || wid(n.p1) != W) fail(MG_E_INVALID, "select lazy default");
              dflt = val(n.p1, i);
              out.coord_lazy[n.p0] = n.p1;
            } else {
              dflt = new_vid(W);
              emit(K_COORD, W, dflt, NONE, NONE, NONE, n.p0, out.coord_row[n.p0]);
            }
            cur = new_vid(W);
            size_t at = emit(K_LOOKUP, W, cur, key, wid(n.b), 0, dflt, 0);
            auto& prior = table_sites[A.table];
            for (auto& pr : prior) {
              if (vwidth[pr.first] != wid(n.b)) continue;  // same name, other sort: separate table
              if (distinct_literals(key, pr.first)) continue;
              code[at].prior.push_back(pr.first);
              code[at].prior.push_back(pr.second);
            }
            code[at].c = (uint32_t)(code[at].prior.size() / 2);
            prior.emplace_back(key, cur);
            site_base_vid[n.p0] = cur;
          } else {
            if (n.p0 != NONE || n.p1 != NONE) fail(MG_E_INVALID, "select over K() has no site");
            cur = val(A.default_node, i);
          }
          for (auto& st : A.stores) {
            uint32_t e = new_vid(1);
            uint32_t si = val(st.first, i);
            emit(K_EQ, 1, e, key, si, NONE, 0, wid(n.b));
            uint32_t sv = val(st.second, i);
            uint32_t nv = new_vid(W);
            emit(K_ITE, W, nv, e, sv, cur, 0, W);
            cur = nv;
          }
          vid[i] = cur;
          break;
        }
        case MG_OP_UFAPP: {
          uint32_t key = val(n.a, i);
          if (n.p0 >= n_tables || tables[n.p0].kind != MG_TABLE_UF) fail(MG_E_INVALID, "uf table");
          if (tables[n.p0].kw != wid(n.a) || tables[n.p0].vw != W) fail(MG_E_INVALID, "uf sorts");
          if (n.p1 >= n_coords || coords[n.p1].kind != MG_COORD_UF_SITE || coords[n.p1].width != W)
            fail(MG_E_INVALID, "uf site coordinate");
          uint32_t dflt;
          if (n.p2 != NONE) {
            dflt = val(n.p2, i);
            if (wid(n.p2) != W) fail(MG_E_INVALID, "lazy default width");
            out.coord_lazy[n.p1] = n.p2;
          } else {
            dflt = new_vid(W);
            emit(K_COORD, W, dflt, NONE, NONE, NONE, n.p1, out.coord_row[n.p1]);
          }
          uint32_t v = new_vid(W);
          size_t at = emit(K_LOOKUP, W, v, key, wid(n.a), 0, dflt, 0);
          auto& prior = table_sites[n.p0];
          for (auto& pr : prior) {
            if (distinct_literals(key, pr.first)) continue;
            code[at].prior.push_back(pr.first);
            code[at].prior.push_back(pr.second);
          }
          code[at].c = (uint32_t)(code[at].prior.size() / 2);
          prior.emplace_back(key, v);
          site_base_vid[n.p1] = v;
          vid[i] = v;
          break;
        }
        case MG_OP_KECCAK: {
          if (W != 256) fail(MG_E_INVALID, "keccak width");
          uint32_t a = NONE;
          if (n.a == NONE) {
            if (n.p0 != 0) fail(MG_E_INVALID, "keccak empty input");
          } else {
            a = val(n.a, i);
            if ((uint64_t)wid(n.a) != 8ull * n.p0 || n.p0 == 0) fail(MG_E_INVALID, "keccak length");
          }
          vid[i] = new_vid(256);
          emit(K_KECCAK, 256, vid[i], a, NONE, NONE, n.p0, 0);
          break;
        }
        default:
          fail(MG_E_UNSUPPORTED, "operator");
      }
      if (root_of[i]) {
        if (is_arr[i] || W != 1) fail(MG_E_INVALID, "root is not Bool");
        emit(K_ASSERT, 1, NONE, val(i, i + 1));
      }
    }
    // watch list (after all nodes: watch entries refer to nodes or site bases); every
    // K_WATCH goes right after the instruction defining its value (one merge pass)
    std::vector<int64_t> def_at(vwidth.size(), -1);
    for (size_t k = 0; k < code.size(); k++)
      if (code[k].dst != NONE && code[k].dst < def_at.size() && def_at[code[k].dst] < 0) def_at[code[k].dst] = (int64_t)k;
    std::vector<std::vector<VInstr>> after(code.size() + 1);
    for (uint64_t j = 0; j < n_watch; j++) {
      uint32_t wv = watch[j];
      uint32_t v, width;
      int64_t at;
      if (wv & 0x80000000u) {
        uint32_t c = wv & 0x7FFFFFFFu;
        if (c >= n_coords || site_base_vid[c] == NONE) fail(MG_E_INVALID, "watch site");
        v = site_base_vid[c];
        width = vwidth[v];
        at = def_at[v];
      } else {
        if (wv >= n_nodes || is_arr[wv]) fail(MG_E_INVALID, "watch node");
        width = nodes[wv].width;
        if (node_const[wv] != NONE) {
          v = new_vid(width);
          def_at.push_back(-1);
          after[code.size()].push_back(VInstr{K_CONST, width, v, NONE, NONE, NONE, node_const[wv], 0, {}});
          at = (int64_t)code.size();  // a rematerialised literal: appended at the end
        } else {
          v = vid[wv];
          at = def_at[v];
        }
      }
      watch_row[j] = wrow;
      after[at < 0 ? code.size() : (size_t)at].push_back(VInstr{K_WATCH, width, NONE, v, NONE, NONE, wrow, 0, {}});
      wrow += L_of(width);
    }
    if (n_watch) {
      std::vector<VInstr> merged;
      merged.reserve(code.size() + 2 * n_watch);
      for (size_t k = 0; k <= code.size(); k++) {
        if (k < code.size()) merged.push_back(std::move(code[k]));
        for (auto& w : after[k]) merged.push_back(std::move(w));
      }
      code.swap(merged);
    }
    out.watch_row = watch_row;
    out.watch_words = wrow;
    out.max_width = max_w;

    // the unlowered program's own slot code only serves explicit-coordinate evaluation on the
    // interpreter (mg_eval; searches run a specialisation): no search over slot orders (for C4's
    // 2,500 instructions that search took two thirds of the lowering)
    allocate(code, vwidth, out, nullptr, /*search_orders=*/false);
    return MG_OK;
  } catch (const Fail& f) {
    err = f.msg;
    return f.code;
  } catch (const std::exception& e) {
    err = e.what();
    return MG_E_INVALID;
  }
}

// ---------------------------------------------------------------------------
// specialisation: value ranges, folding, aliases, dead code (specialize_program)
// ---------------------------------------------------------------------------
namespace {

inline uint32_t Lw(uint32_t w) { return (w + 31) / 32; }

// 256-bit unsigned words for the analysis (values of width <= 256; wider values are unknown)
struct U256 {
  uint64_t w[4] = {0, 0, 0, 0};
  static U256 of(uint64_t v) {
    U256 r;
    r.w[0] = v;
    return r;
  }
  // limbs [0, L) of 32 bits; false if a limb at or above 256 bits is nonzero
  static bool from_limbs(const uint32_t* x, uint32_t L, U256* out) {
    U256 r;
    for (uint32_t j = 0; j < L; j++) {
      if (j >= 8) {
        if (x[j]) return false;
        continue;
      }
      r.w[j / 2] |= (uint64_t)x[j] << (32 * (j % 2));
    }
    *out = r;
    return true;
  }
  static U256 ones(uint32_t w) {  // 2^w - 1, w <= 256
    U256 r;
    for (int i = 0; i < 4; i++) {
      const int b = (int)w - 64 * i;
      r.w[i] = b >= 64 ? ~0ull : b <= 0 ? 0ull : ((1ull << b) - 1ull);
    }
    return r;
  }
  bool zero() const { return !(w[0] | w[1] | w[2] | w[3]); }
  bool operator==(const U256& o) const { return !std::memcmp(w, o.w, sizeof(w)); }
  bool operator!=(const U256& o) const { return !(*this == o); }
  bool operator<(const U256& o) const {
    for (int i = 3; i >= 0; i--)
      if (w[i] != o.w[i]) return w[i] < o.w[i];
    return false;
  }
  bool operator<=(const U256& o) const { return !(o < *this); }
  U256 operator&(const U256& o) const { U256 r; for (int i = 0; i < 4; i++) r.w[i] = w[i] & o.w[i]; return r; }
  U256 operator|(const U256& o) const { U256 r; for (int i = 0; i < 4; i++) r.w[i] = w[i] | o.w[i]; return r; }
  U256 operator^(const U256& o) const { U256 r; for (int i = 0; i < 4; i++) r.w[i] = w[i] ^ o.w[i]; return r; }
  U256 operator~() const { U256 r; for (int i = 0; i < 4; i++) r.w[i] = ~w[i]; return r; }
  // sum; *carry = carry out of bit 255
  static U256 add(const U256& a, const U256& b, bool* carry) {
    U256 r;
    unsigned __int128 c = 0;
    for (int i = 0; i < 4; i++) {
      c += (unsigned __int128)a.w[i] + b.w[i];
      r.w[i] = (uint64_t)c;
      c >>= 64;
    }
    if (carry) *carry = c != 0;
    return r;
  }
  static U256 sub(const U256& a, const U256& b) {  // mod 2^256
    U256 r;
    uint64_t br = 0;
    for (int i = 0; i < 4; i++) {
      const unsigned __int128 t = (unsigned __int128)a.w[i] - b.w[i] - br;
      r.w[i] = (uint64_t)t;
      br = (uint64_t)(t >> 64) & 1u;
    }
    return r;
  }
  U256 shr(uint32_t n) const {
    if (n >= 256) return U256{};
    U256 r;
    const uint32_t q = n / 64, s = n % 64;
    for (uint32_t i = 0; i + q < 4; i++) {
      uint64_t v = w[i + q] >> s;
      if (s && i + q + 1 < 4) v |= w[i + q + 1] << (64 - s);
      r.w[i] = v;
    }
    return r;
  }
  U256 shl(uint32_t n) const {  // bits beyond 255 dropped
    if (n >= 256) return U256{};
    U256 r;
    const uint32_t q = n / 64, s = n % 64;
    for (uint32_t i = q; i < 4; i++) {
      uint64_t v = w[i - q] << s;
      if (s && i - q >= 1) v |= w[i - q - 1] >> (64 - s);
      r.w[i] = v;
    }
    return r;
  }
  int top_bit() const {  // index of the highest set bit, -1 if zero
    for (int i = 3; i >= 0; i--)
      if (w[i]) return 64 * i + 63 - __builtin_clzll(w[i]);
    return -1;
  }
  int trailing_ones() const {
    for (int i = 0; i < 4; i++)
      if (~w[i]) return 64 * i + __builtin_ctzll(~w[i]);
    return 256;
  }
};

constexpr size_t kMaxSet = 16;  // value sets (DICT coordinates, constants) up to this many entries

struct Analysis {
  const Lowered& P;
  const std::vector<GenSpec>* specs;
  const std::vector<uint32_t>* gconsts;
  Analysis(const Lowered& p, const std::vector<GenSpec>* s, const std::vector<uint32_t>* g) : P(p), specs(s), gconsts(g) {}
  // Abstract value of an SSA id (widths <= 256; anything wider is unknown), three facts that
  // hold for EVERY candidate the kernel evaluates.  In the search kernel a coordinate's facts
  // come from its generator spec, which bounds every candidate it draws (clamp records,
  // dictionaries, alignment, fixed bits):
  //  * rng: the value lies in [lo, hi];
  //  * known bits: bits in z are 0, bits in o are 1 (bits at or above the width are in z);
  //  * set (has_set): the value is one of at most kMaxSet values (a DICT coordinate, e.g. the
  //    caller drawn from LASER's actors, and what selects or slices of it give).
  // A comparison they decide folds to a literal, an ITE on it becomes an alias of the chosen
  // arm, and bits() then looks through it (e.g. the calldata guard If(k < size, calldata[k], 0)
  // with size drawn from [68, 2^32) collapses to the byte, and a CALLDATALOAD to its AUX word).
  struct Rng {
    bool k = false;
    U256 lo, hi;
  };
  struct KB {
    bool k = false;
    U256 z, o;
  };
  struct Val {
    Rng r;
    KB kb;
    bool has_set = false;
    std::vector<U256> set;  // sorted, unique
  };
  // A Bool that equals (src in S), or its negation: the disjunction Or(x == c1, x == c2, ...)
  // LASER builds for the caller of every transaction is one; when src's own set lies inside S
  // (or outside it) the predicate is decided.
  struct Mem {
    bool k = false, neg = false;
    uint32_t src = 0;
    std::vector<U256> S;
  };
  std::vector<Val> val;
  std::vector<Mem> mem;
  // psrc/plo: the value is bits [plo, plo + width) of value psrc (a chain of EXTRACTs, and
  // CONCATs of adjacent slices of one value, e.g. a CALLDATALOAD of an AUX word's bytes)
  std::vector<uint32_t> psrc, plo;
  std::vector<int8_t> fold;       // per id: -1, or the folded Bool value
  std::vector<uint32_t> alias;    // per id: the id it equals (itself if none)
  std::vector<char> skip;         // per instruction: defines an alias / a decided assert
  std::vector<Val> cval;          // per coordinate (search mode)
  std::vector<int32_t> defk;      // per id: index of its defining instruction (-1: none)
  std::map<size_t, Instr> rewrite;  // instruction index -> the instruction emitted instead
  // LOOKUP instruction index -> (default, (key, value) pairs) after pruning
  std::map<size_t, std::pair<uint32_t, std::vector<uint32_t>>> lookup_rw;
  std::map<std::vector<uint32_t>, uint32_t> lit_id;  // literal (limbs, width) -> its first value id
  // segs[id]: the value as slices of other values, low bits first (empty: see segs_of)
  struct Seg {
    uint32_t src, lo, w;
  };
  static constexpr size_t kMaxSegs = 4;
  std::vector<std::vector<Seg>> segs;
  std::vector<Seg> segs_of(uint32_t id) const {
    id = res(id);
    if (!segs[id].empty()) return segs[id];
    if (psrc[id] != MG_NONE) return {Seg{psrc[id], plo[id], P.vwidth[id]}};
    return {Seg{id, 0, P.vwidth[id]}};
  }
  static void seg_push(std::vector<Seg>& v, const Seg& x) {
    if (!v.empty() && v.back().src == x.src && v.back().lo + v.back().w == x.lo) v.back().w += x.w;
    else v.push_back(x);
  }

  uint32_t res(uint32_t id) const {
    if (alias.empty() || id >= alias.size()) return id;
    while (alias[id] != id) id = alias[id];
    return id;
  }

  // ---- lattice helpers ----
  static Rng rfull(uint32_t w) {
    Rng r;
    if (w <= 256) {
      r.k = true;
      r.hi = U256::ones(w);
    }
    return r;
  }
  static Rng rexact(const U256& v) {
    Rng r;
    r.k = true;
    r.lo = r.hi = v;
    return r;
  }
  static Rng rhull(const Rng& a, const Rng& b) {
    Rng r;
    if (!a.k || !b.k) return r;
    r.k = true;
    r.lo = a.lo < b.lo ? a.lo : b.lo;
    r.hi = a.hi < b.hi ? b.hi : a.hi;
    return r;
  }
  static KB kfull(uint32_t w) {
    KB k;
    if (w <= 256) {
      k.k = true;
      k.z = ~U256::ones(w);
    }
    return k;
  }
  static KB kexact(const U256& v, uint32_t w) {
    KB k;
    k.k = true;
    k.o = v;
    k.z = ~v;
    (void)w;
    return k;
  }
  static KB kmeet(const KB& a, const KB& b) {
    KB k;
    if (!a.k || !b.k) return k;
    k.k = true;
    k.z = a.z & b.z;
    k.o = a.o & b.o;
    return k;
  }
  static Val vfull(uint32_t w) {
    Val v;
    v.r = rfull(w);
    v.kb = kfull(w);
    return v;
  }
  static Val vexact(const U256& x, uint32_t w) {
    Val v;
    v.r = rexact(x);
    v.kb = kexact(x, w);
    v.has_set = true;
    v.set = {x};
    return v;
  }
  static void set_norm(std::vector<U256>& s) {
    std::sort(s.begin(), s.end());
    s.erase(std::unique(s.begin(), s.end()), s.end());
  }
  static bool exact_of(const Val& v, U256* x) {
    if (v.r.k && v.r.lo == v.r.hi) {
      *x = v.r.lo;
      return true;
    }
    return false;
  }
  // tighten: range from known bits and known bits from range; a set tightens both
  static void tighten(Val& v, uint32_t w) {
    if (w > 256) {
      v = Val{};
      return;
    }
    if (!v.r.k) v.r = rfull(w);
    if (!v.kb.k) v.kb = kfull(w);
    const U256 m = U256::ones(w);
    v.kb.z = v.kb.z | ~m;
    v.kb.o = v.kb.o & m;
    if (v.has_set) {
      if (v.set.empty() || v.set.size() > kMaxSet) {
        v.has_set = false;
        v.set.clear();
      } else {
        Rng h = rexact(v.set[0]);
        KB kk = kexact(v.set[0], w);
        for (const U256& x : v.set) {
          h = rhull(h, rexact(x));
          kk = kmeet(kk, kexact(x, w));
        }
        v.r = h;  // the set's hull is inside any other range fact we hold
        v.kb.z = v.kb.z | kk.z;
        v.kb.o = v.kb.o | kk.o;
      }
    }
    // bits above the highest bit of hi are zero; the common prefix of lo and hi is known
    const int d = (v.r.lo ^ v.r.hi).top_bit();
    const U256 above = d >= 255 ? U256{} : ~U256::ones((uint32_t)(d + 1));
    v.kb.z = v.kb.z | (above & ~v.r.lo);
    v.kb.o = v.kb.o | (above & v.r.lo);
    // range from known bits: lo >= ones, hi <= not-zeros
    const U256 klo = v.kb.o, khi = ~v.kb.z & m;
    if (v.r.lo < klo) v.r.lo = klo;
    if (khi < v.r.hi) v.r.hi = khi;
    if (v.r.hi < v.r.lo) {  // contradictory facts cannot happen for reachable values; stay safe
      v.r = rfull(w);
      v.kb = kfull(w);
      v.has_set = false;
      v.set.clear();
    }
  }

  // value of a generated coordinate (include/mythgpu.h GEN3)
  Val coord_val(uint32_t c) const {
    const GenSpec& sp = (*specs)[c];
    const uint32_t w = P.coord_width[c], L = Lw(w), kind = sp.kind & 0xFFu;
    Val v;
    if (w > 256) return v;
    const auto& G = *gconsts;
    const U256 wlim = U256::ones(w);
    auto lim = [&](uint32_t off, U256* x) { return U256::from_limbs(&G[off], L, x); };
    switch (kind) {
      case MG_GEN_FIXED: {
        U256 x;
        if (lim(sp.p[0], &x)) v = vexact(x, w);
        break;
      }
      case MG_GEN_DICT:
      case MG_GEN_MIXED: {
        std::vector<U256> d;  // dictionary entries
        bool ok = sp.p[1] > 0;
        for (uint32_t e = 0; ok && e < sp.p[1]; e++) {
          U256 x;
          if (!lim(sp.p[0] + e * L, &x)) ok = false;
          else d.push_back(x);
        }
        Rng dh;
        if (ok) {
          dh = rexact(d[0]);
          for (const U256& x : d) dh = rhull(dh, rexact(x));
        }
        if (kind == MG_GEN_DICT) {
          if (ok) {
            v.r = dh;
            if (d.size() <= kMaxSet) {
              v.has_set = true;
              v.set = d;
              set_norm(v.set);
            }
          }
          break;
        }
        if (sp.p[6]) {  // clamp record: the final value is inside [lo, lo + span)
          U256 lo;
          const uint32_t rec = sp.p[6] - 1;
          if (lim(rec, &lo)) {
            const uint64_t span = G[rec + L] ? G[rec + L] : (1ull << 32);
            bool cy = false;
            const U256 hi = U256::add(lo, U256::of(span - 1), &cy);
            if (!cy && hi <= wlim) {
              v.r.k = true;
              v.r.lo = lo;
              v.r.hi = hi;
            }
          }
          break;
        }
        const uint32_t pc = sp.p[3] != MG_NONE ? (sp.p[2] & 0xFFFFu) : 0u;
        const uint32_t pd = sp.p[1] ? (sp.p[2] >> 16) : 0u;
        const uint32_t ps = sp.p[4] & 0xFFFFu;
        Rng u;
        bool have = false, unknown = false;
        auto add = [&](const Rng& x) {
          if (!x.k) unknown = true;
          else u = have ? rhull(u, x) : x;
          have = true;
        };
        Rng cd;  // COPY / DICT part, before the delta
        bool cd_have = false, cd_unknown = false;
        if (pc) {
          const Rng s = cval[sp.p[3]].r;
          if (!s.k) cd_unknown = true;
          else cd = s;
          cd_have = true;
        }
        if (pd) {
          if (!ok) cd_unknown = true;
          else cd = cd_have && cd.k ? rhull(cd, dh) : dh;
          cd_have = true;
        }
        if (cd_have) {
          if (cd_unknown) {
            add(Rng{});
          } else if (sp.p[5]) {  // +/-2 at most, no wrap
            bool cy = false;
            const U256 hi2 = U256::add(cd.hi, U256::of(2), &cy);
            if (U256::of(2) <= cd.lo && !cy && hi2 <= wlim) {
              Rng x;
              x.k = true;
              x.lo = U256::sub(cd.lo, U256::of(2));
              x.hi = hi2;
              add(x);
            } else {
              add(rfull(w));
            }
          } else {
            add(cd);
          }
        }
        const uint32_t sb = std::min(w, sp.p[4] >> 16);
        if (ps) add(rfull(sb));
        if (pc + pd + ps < 65536u) add(rfull(w));
        if (have && !unknown) v.r = u;
        break;
      }
      case MG_GEN_RANGE: {
        U256 lo;
        if (lim(sp.p[0], &lo)) {
          const uint64_t span = sp.p[1] ? sp.p[1] : (1ull << 32);
          bool cy = false;
          const U256 hi = U256::add(lo, U256::of(span - 1), &cy);
          if (!cy && hi <= wlim) {
            v.r.k = true;
            v.r.lo = lo;
            v.r.hi = hi;
          }
        }
        break;
      }
      case MG_GEN_ALIGNED: {
        U256 lo;
        if (lim(sp.p[0], &lo) && sp.p[1] < 256) {
          const uint64_t cnt = sp.p[2] ? sp.p[2] : (1ull << 32);
          const U256 step = U256::of(cnt - 1).shl(sp.p[1]);
          bool cy = false;
          const U256 top = U256::add(lo, step, &cy);
          // (cnt - 1) << p1 must not lose bits either
          if (!cy && top <= wlim && step.shr(sp.p[1]) == U256::of(cnt - 1)) {
            v.r.k = true;
            v.r.lo = lo;
            v.r.hi = top;
          }
          // lo + (m << p1): the low p1 bits are lo's, wrap or not
          v.kb = kfull(w);
          const U256 low = U256::ones(std::min(sp.p[1], w));
          v.kb.z = v.kb.z | (low & ~lo);
          v.kb.o = lo & low;
        }
        break;
      }
      default:  // UNIFORM / LAZY
        break;
    }
    tighten(v, w);
    if (const uint32_t fix = sp.kind >> 8) {  // (v & ~m) | val
      U256 m, fv;
      if (U256::from_limbs(&G[fix - 1], L, &m) && U256::from_limbs(&G[fix - 1 + L], L, &fv)) {
        m = m & wlim;
        fv = fv & m;
        Val f;
        f.kb.k = true;
        f.kb.z = (v.kb.z & ~m) | (m & ~fv);
        f.kb.o = (v.kb.o & ~m) | fv;
        if (v.has_set) {
          f.has_set = true;
          for (const U256& x : v.set) f.set.push_back((x & ~m) | fv);
          set_norm(f.set);
        }
        v = f;
        tighten(v, w);
      } else {
        v = vfull(w);
      }
    }
    return v;
  }

  // decide a comparison from the operands' facts: -1 undecided, else 0 / 1
  static int decide(uint32_t op, const Val& a, const Val& b, uint32_t wa) {
    if (wa > 256 || !a.r.k || !b.r.k) return -1;
    if (op == K_EQ) {
      U256 x, y;
      if (exact_of(a, &x) && exact_of(b, &y)) return x == y;
      if (a.r.hi < b.r.lo || b.r.hi < a.r.lo) return 0;
      if (a.kb.k && b.kb.k && !((a.kb.o & b.kb.z) | (a.kb.z & b.kb.o)).zero()) return 0;
      if (a.has_set && b.has_set) {
        bool any = false;
        for (const U256& p : a.set)
          if (std::binary_search(b.set.begin(), b.set.end(), p)) any = true;
        if (!any) return 0;
      }
      return -1;
    }
    Rng ra = a.r, rb = b.r;
    if (op == K_SLT || op == K_SLE) {
      // both non-negative (sign bit known zero): signed order is unsigned order
      const U256 sign = U256::of(1).shl(wa - 1);
      if (sign <= ra.hi || sign <= rb.hi) return -1;
      op = op == K_SLT ? K_ULT : K_ULE;
    }
    switch (op) {
      case K_ULT:
        if (ra.hi < rb.lo) return 1;
        if (rb.hi <= ra.lo) return 0;
        return -1;
      case K_ULE:
        if (ra.hi <= rb.lo) return 1;
        if (rb.hi < ra.lo) return 0;
        return -1;
      default:
        return -1;
    }
  }

  // x == y decided from the facts, looking through CONCATs of equal split (keys of 512 bits and
  // more, e.g. Concat(address, slot) of a keccak site): -1 undecided, else 0 / 1
  int decide_eq(uint32_t x, uint32_t y, uint32_t w, int depth = 0) const {
    x = res(x);
    y = res(y);
    if (x == y) return 1;
    if (w <= 256) {
      const int v = decide(K_EQ, val[x], val[y], w);
      if (v >= 0 || depth > 8) return v;
    }
    if (depth > 8) return -1;
    const int32_t kx = defk[x], ky = defk[y];
    if (kx < 0 || ky < 0) return -1;
    const Instr &dx = P.vcode[kx], &dy = P.vcode[ky];
    if (dx.op != K_CONCAT || dy.op != K_CONCAT || dx.p1 != dy.p1) return -1;
    const int lo = decide_eq(dx.b, dy.b, dx.p1, depth + 1);
    if (lo == 0) return 0;
    const int hi = decide_eq(dx.a, dy.a, w - dx.p1, depth + 1);
    if (hi == 0) return 0;
    return lo == 1 && hi == 1 ? 1 : -1;
  }

  int decide_mem(const Mem& m) const {
    if (!m.k) return -1;
    const Val& s = val[res(m.src)];
    if (!s.has_set) return -1;
    size_t in = 0;
    for (const U256& x : s.set)
      if (std::binary_search(m.S.begin(), m.S.end(), x)) in++;
    int v = -1;
    if (in == s.set.size()) v = 1;
    else if (in == 0) v = 0;
    if (v >= 0 && m.neg) v = 1 - v;
    return v;
  }

  void analyze(bool search) {
    const size_t nv = P.vwidth.size();
    val.assign(nv, Val{});
    mem.assign(nv, Mem{});
    psrc.assign(nv, MG_NONE);
    plo.assign(nv, 0);
    fold.assign(nv, -1);
    alias.resize(nv);
    for (size_t i = 0; i < nv; i++) alias[i] = (uint32_t)i;
    skip.assign(P.vcode.size(), 0);
    defk.assign(nv, -1);
    rewrite.clear();
    lookup_rw.clear();
    lit_id.clear();
    segs.assign(nv, {});
    for (size_t k = 0; k < P.vcode.size(); k++)
      if (P.vcode[k].dst < nv && defk[P.vcode[k].dst] < 0) defk[P.vcode[k].dst] = (int32_t)k;
    if (search && specs) {
      cval.assign(P.n_coords, Val{});
      for (uint32_t c = 0; c < P.n_coords; c++) cval[c] = coord_val(c);
    }
    for (size_t k = 0; k < P.vcode.size(); k++) {
      const Instr& in = P.vcode[k];
      const uint32_t d = in.dst, W = in.wd;
      auto V = [&](uint32_t id) -> const Val& { return val[res(id)]; };
      auto F = [&](uint32_t id) { return (int)fold[res(id)]; };
      auto alias_to = [&](uint32_t src) {
        alias[d] = res(src);
        val[d] = val[res(src)];
        mem[d] = mem[res(src)];
        fold[d] = fold[res(src)];
        skip[k] = 1;
      };
      auto set_fold = [&](int v) {
        fold[d] = (int8_t)v;
        val[d] = vexact(U256::of((uint64_t)v), 1);
      };
      if (d == MG_NONE || d >= nv) {
        if (in.op == K_ASSERT && F(in.a) == 1) skip[k] = 1;
        continue;
      }
      Val r = vfull(W);
      switch (in.op) {
        case K_CONST: {
          {  // one value per literal: later copies alias the first (no reload in the interpreter, and
             // rewrites that match operands by id see equal literals as equal)
            std::vector<uint32_t> key(P.consts.begin() + in.p0, P.consts.begin() + in.p0 + Lw(W));
            key.push_back(W);
            auto it = lit_id.find(key);
            if (it != lit_id.end()) {
              alias_to(it->second);
              continue;
            }
            lit_id.emplace(std::move(key), d);
          }
          U256 x;
          if (W <= 256 && U256::from_limbs(&P.consts[in.p0], Lw(W), &x)) r = vexact(x & U256::ones(W), W);
          if (W == 1 && r.r.k) fold[d] = (int8_t)(r.r.lo.w[0] & 1u);  // a Bool literal (e.g. a folded root)
          break;
        }
        case K_COORD:
          if (search && specs) r = cval[in.p0];
          break;
        case K_COPY:
          alias_to(in.a);
          continue;
        case K_ZEXT: {
          const Val& a = V(in.a);
          if (W <= 256 && in.p1 <= 256) {
            r = a;
            if (!r.r.k) r.r = rfull(in.p1);
            if (!r.kb.k) r.kb = kfull(in.p1);
          }
          break;
        }
        case K_SEXT: {
          const Val& a = V(in.a);
          const uint32_t wa = in.p1;
          if (W <= 256 && wa <= 256 && a.kb.k) {
            const U256 sign = U256::of(1).shl(wa - 1);
            const U256 ext = U256::ones(W) & ~U256::ones(wa);
            if (!(a.kb.z & sign).zero()) {  // non-negative: a zero extension
              r = a;
            } else if (!(a.kb.o & sign).zero()) {  // negative: high bits ones
              r.kb.k = true;
              r.kb.z = a.kb.z & U256::ones(wa);
              r.kb.o = a.kb.o | ext;
              r.r = rfull(W);
            }
          }
          break;
        }
        case K_EXTRACT: {
          const Val& a = V(in.a);
          const uint32_t wa = in.p1;
          if (W <= 256 && wa <= 256) {
            const U256 m = U256::ones(W);
            if (a.r.k && a.r.hi.shr(in.p0) <= m) {
              r.r.k = true;
              r.r.lo = a.r.lo.shr(in.p0);
              r.r.hi = a.r.hi.shr(in.p0);
            }
            if (a.kb.k) {
              r.kb.k = true;
              r.kb.z = a.kb.z.shr(in.p0) | ~m;
              r.kb.o = a.kb.o.shr(in.p0) & m;
            }
            if (a.has_set) {
              r.has_set = true;
              for (const U256& x : a.set) r.set.push_back(x.shr(in.p0) & m);
              set_norm(r.set);
            }
          }
          const uint32_t ra = res(in.a);
          std::vector<Seg> sl;  // the slice [p0, p0 + W) of a's segments
          {
            uint32_t pos = 0;
            for (const Seg& sg : segs_of(ra)) {
              const uint32_t lo = std::max(pos, in.p0), hi = std::min(pos + sg.w, in.p0 + W);
              if (lo < hi) seg_push(sl, Seg{sg.src, sg.lo + (lo - pos), hi - lo});
              pos += sg.w;
            }
          }
          if (sl.size() == 1) {  // bits of one value (through EXTRACTs and CONCATs of its slices)
            if (sl[0].lo == 0 && W == P.vwidth[sl[0].src]) {
              alias_to(sl[0].src);
              continue;
            }
            psrc[d] = sl[0].src;
            plo[d] = sl[0].lo;
          } else {
            psrc[d] = ra;
            plo[d] = in.p0;
            if (sl.size() <= kMaxSegs) segs[d] = std::move(sl);
          }
          break;
        }
        case K_CONCAT: {
          {  // adjacent slices of one value: the high part starts where the low part ends
            const uint32_t ra = res(in.a), rb = res(in.b);
            const uint32_t sa = psrc[ra] != MG_NONE ? psrc[ra] : ra, la = psrc[ra] != MG_NONE ? plo[ra] : 0u;
            const uint32_t sb = psrc[rb] != MG_NONE ? psrc[rb] : rb, lb = psrc[rb] != MG_NONE ? plo[rb] : 0u;
            if (sa == sb && la == lb + P.vwidth[rb]) {
              if (lb == 0 && W == P.vwidth[sa]) {
                alias_to(sa);
                continue;
              }
              psrc[d] = sa;
              plo[d] = lb;
              r = vfull(W);
              break;
            }
          }
          {  // a chain of concatenated slices (e.g. a word rebuilt byte by byte from another word,
             // Concat(x, Extract(255, 248, y), ..., Extract(7, 0, y))): merged segments; when they are
             // two whole values the chain is one CONCAT of them
            std::vector<Seg> sg = segs_of(in.b);
            for (const Seg& x : segs_of(in.a)) seg_push(sg, x);
            auto whole = [&](const Seg& x) { return x.lo == 0 && x.w == P.vwidth[x.src]; };
            if (sg.size() == 1) {
              if (whole(sg[0])) {
                alias_to(sg[0].src);
                continue;
              }
              psrc[d] = sg[0].src;
              plo[d] = sg[0].lo;
              r = vfull(W);
              break;
            }
            if (sg.size() == 2 && whole(sg[0]) && whole(sg[1]) && (sg[0].src != res(in.b) || sg[1].src != res(in.a)))
              rewrite[k] = Instr{K_CONCAT, W, d, sg[1].src, sg[0].src, MG_NONE, 0, sg[0].w};
            if (sg.size() <= kMaxSegs) segs[d] = std::move(sg);
          }
          const Val &a = V(in.a), &b = V(in.b);
          const uint32_t wb = in.p1;
          if (W <= 256 && a.r.k && b.r.k) {
            r.r.k = true;  // a * 2^wb + b, b < 2^wb
            r.r.lo = a.r.lo.shl(wb) | b.r.lo;
            r.r.hi = a.r.hi.shl(wb) | b.r.hi;
          }
          if (W <= 256 && a.kb.k && b.kb.k) {
            r.kb.k = true;
            r.kb.z = a.kb.z.shl(wb) | (b.kb.z & U256::ones(wb)) | ~U256::ones(W);
            r.kb.o = a.kb.o.shl(wb) | (b.kb.o & U256::ones(wb));
          }
          if (W <= 256 && a.has_set && b.has_set && a.set.size() * b.set.size() <= kMaxSet) {
            r.has_set = true;
            for (const U256& x : a.set)
              for (const U256& y : b.set) r.set.push_back(x.shl(wb) | y);
            set_norm(r.set);
          }
          break;
        }
        case K_AND:
        case K_OR:
        case K_XOR: {
          if (in.op != K_XOR && res(in.a) == res(in.b)) {  // x & x = x | x = x
            alias_to(in.a);
            continue;
          }
          const int fa = F(in.a), fb = F(in.b);
          if (W == 1) {
            if (in.op == K_AND) {
              if (fa == 0 || fb == 0) { set_fold(0); continue; }
              if (fa == 1) { alias_to(in.b); continue; }
              if (fb == 1) { alias_to(in.a); continue; }
            } else if (in.op == K_OR) {
              if (fa == 1 || fb == 1) { set_fold(1); continue; }
              if (fa == 0) { alias_to(in.b); continue; }
              if (fb == 0) { alias_to(in.a); continue; }
            } else if (fa >= 0 && fb >= 0) {
              set_fold(fa ^ fb);
              continue;
            }
            // membership predicates over one value: Or = union, And = intersection
            const Mem &ma = mem[res(in.a)], &mb = mem[res(in.b)];
            if (in.op != K_XOR && ma.k && mb.k && res(ma.src) == res(mb.src) && ma.neg == mb.neg) {
              Mem m;
              m.k = true;
              m.src = res(ma.src);
              m.neg = ma.neg;
              // Or of positives = union; And of positives = intersection (negated: De Morgan)
              const bool uni = (in.op == K_OR) != ma.neg;
              if (uni) {
                m.S = ma.S;
                m.S.insert(m.S.end(), mb.S.begin(), mb.S.end());
                set_norm(m.S);
              } else {
                for (const U256& x : ma.S)
                  if (std::binary_search(mb.S.begin(), mb.S.end(), x)) m.S.push_back(x);
              }
              const int v = decide_mem(m);
              if (v >= 0) { set_fold(v); continue; }
              mem[d] = m;
            }
            // Or(a < b, a == b) is a <= b: LASER's ULE/UGE/SLE/SGE (mythril/laser/smt/bitvec_helper.py:53-80,
            // Or(ULT(a, b), a == b)) as one borrow chain instead of a chain plus an equality
            if (in.op == K_OR) {
              auto def = [&](uint32_t id) -> const Instr* {
                const int32_t x = defk[res(id)];
                return x >= 0 && !skip[x] ? &P.vcode[x] : nullptr;
              };
              const Instr *x = def(in.a), *y = def(in.b);
              if (x && y && x->op == K_EQ) std::swap(x, y);
              if (x && y && y->op == K_EQ && (x->op == K_ULT || x->op == K_SLT) && x->p1 == y->p1) {
                const uint32_t xa = res(x->a), xb = res(x->b), ya = res(y->a), yb = res(y->b);
                if ((xa == ya && xb == yb) || (xa == yb && xb == ya)) {
                  rewrite[k] = Instr{x->op == K_ULT ? (uint32_t)K_ULE : (uint32_t)K_SLE, 1, d, x->a, x->b, MG_NONE, 0, x->p1};
                }
              }
            }
            break;
          }
          const Val &a = V(in.a), &b = V(in.b);
          if (W <= 256 && a.kb.k && b.kb.k) {
            r.kb.k = true;
            if (in.op == K_AND) {
              r.kb.z = a.kb.z | b.kb.z;
              r.kb.o = a.kb.o & b.kb.o;
            } else if (in.op == K_OR) {
              r.kb.z = a.kb.z & b.kb.z;
              r.kb.o = a.kb.o | b.kb.o;
            } else {
              const U256 kn = (a.kb.z | a.kb.o) & (b.kb.z | b.kb.o), x = a.kb.o ^ b.kb.o;
              r.kb.z = kn & ~x;
              r.kb.o = kn & x;
            }
            r.r = rfull(W);
          }
          if (W <= 256 && a.has_set && b.has_set && a.set.size() * b.set.size() <= kMaxSet) {
            r.has_set = true;
            for (const U256& x : a.set)
              for (const U256& y : b.set) r.set.push_back(in.op == K_AND ? (x & y) : in.op == K_OR ? (x | y) : (x ^ y));
            set_norm(r.set);
          }
          break;
        }
        case K_NOT:
          if (W == 1) {
            if (F(in.a) >= 0) {
              set_fold(1 - F(in.a));
              continue;
            }
            const Mem& ma = mem[res(in.a)];
            if (ma.k) {
              mem[d] = ma;
              mem[d].neg = !ma.neg;
            }
            break;
          }
          if (W <= 256) {
            const Val& a = V(in.a);
            const U256 m = U256::ones(W);
            if (a.kb.k) {
              r.kb.k = true;
              r.kb.z = a.kb.o | ~m;
              r.kb.o = a.kb.z & m;
            }
            if (a.has_set) {
              r.has_set = true;
              for (const U256& x : a.set) r.set.push_back(~x & m);
              set_norm(r.set);
            }
          }
          break;
        case K_ITE: {
          const int fc = F(in.a);
          if (fc >= 0) {
            alias_to(fc ? in.b : in.c);
            continue;
          }
          if (res(in.b) == res(in.c)) {
            alias_to(in.b);
            continue;
          }
          const Val &b = V(in.b), &c = V(in.c);
          if (W <= 256) {
            r.r = rhull(b.r, c.r);
            r.kb = kmeet(b.kb, c.kb);
            if (b.has_set && c.has_set) {
              r.has_set = true;
              r.set = b.set;
              r.set.insert(r.set.end(), c.set.begin(), c.set.end());
              set_norm(r.set);
            }
          }
          break;
        }
        case K_ADD: {
          const Val &a = V(in.a), &b = V(in.b);
          if (W <= 256 && a.r.k && b.r.k) {
            bool cy = false;
            const U256 hi = U256::add(a.r.hi, b.r.hi, &cy);
            if (!cy && hi <= U256::ones(W)) {
              r.r.lo = U256::add(a.r.lo, b.r.lo, nullptr);
              r.r.hi = hi;
            }
          }
          if (W <= 256 && a.kb.k && b.kb.k) {  // low bits known in both operands: known sum
            const int t = std::min((a.kb.z | a.kb.o).trailing_ones(), (b.kb.z | b.kb.o).trailing_ones());
            if (t > 0) {
              const U256 lm = U256::ones((uint32_t)std::min(t, (int)W));
              const U256 s = U256::add(a.kb.o & lm, b.kb.o & lm, nullptr) & lm;
              r.kb.z = r.kb.z | (lm & ~s);
              r.kb.o = r.kb.o | s;
            }
          }
          if (W <= 256 && a.has_set && b.has_set && a.set.size() * b.set.size() <= kMaxSet) {
            r.has_set = true;
            for (const U256& x : a.set)
              for (const U256& y : b.set) r.set.push_back(U256::add(x, y, nullptr) & U256::ones(W));
            set_norm(r.set);
          }
          break;
        }
        case K_SUB: {
          const Val &a = V(in.a), &b = V(in.b);
          if (W <= 256 && a.r.k && b.r.k && b.r.hi <= a.r.lo) {
            r.r.lo = U256::sub(a.r.lo, b.r.hi);
            r.r.hi = U256::sub(a.r.hi, b.r.lo);
          }
          if (W <= 256 && a.kb.k && b.kb.k) {
            const int t = std::min((a.kb.z | a.kb.o).trailing_ones(), (b.kb.z | b.kb.o).trailing_ones());
            if (t > 0) {
              const U256 lm = U256::ones((uint32_t)std::min(t, (int)W));
              const U256 s = U256::sub(a.kb.o & lm, b.kb.o & lm) & lm;
              r.kb.z = r.kb.z | (lm & ~s);
              r.kb.o = r.kb.o | s;
            }
          }
          if (W <= 256 && a.has_set && b.has_set && a.set.size() * b.set.size() <= kMaxSet) {
            r.has_set = true;
            for (const U256& x : a.set)
              for (const U256& y : b.set) r.set.push_back(U256::sub(x, y) & U256::ones(W));
            set_norm(r.set);
          }
          break;
        }
        case K_EQ:
        case K_ULT:
        case K_ULE:
        case K_SLT:
        case K_SLE: {
          const Val &a = V(in.a), &b = V(in.b);
          int v = in.op == K_EQ ? decide_eq(in.a, in.b, in.p1) : decide(in.op, a, b, in.p1);
          if (v < 0 && res(in.a) == res(in.b)) v = (in.op == K_ULT || in.op == K_SLT) ? 0 : 1;  // x op x
          if (v >= 0) {
            set_fold(v);
            continue;
          }
          if (in.op == K_EQ) {  // x == c: a membership predicate {c} over x
            U256 c;
            uint32_t x = MG_NONE;
            if (exact_of(b, &c)) x = res(in.a);
            else if (exact_of(a, &c)) x = res(in.b);
            if (x != MG_NONE) {
              Mem m;
              m.k = true;
              m.src = x;
              m.S = {c};
              const int dv = decide_mem(m);
              if (dv >= 0) { set_fold(dv); continue; }
              mem[d] = m;
            }
          }
          r = vfull(1);
          break;
        }
        case K_LOOKUP: {
          if (in.c == 0) {  // no earlier site can share the key: the default
            alias_to(in.p0);
            continue;
          }
          // priors whose key can never equal this key are dropped; a prior whose key always
          // equals it ends the list and becomes the default (first match wins)
          std::vector<uint32_t> kept;  // (key, value) pairs
          uint32_t dflt = in.p0;
          for (uint32_t p = 0; p < in.c; p++) {
            const uint32_t kv = P.vaux[in.p1 + 2 * p], vv = P.vaux[in.p1 + 2 * p + 1];
            const int e = decide_eq(in.a, kv, in.b);
            if (e == 0) continue;
            if (e == 1) {
              dflt = vv;
              break;
            }
            kept.push_back(kv);
            kept.push_back(vv);
          }
          if (kept.empty()) {
            alias_to(dflt);
            continue;
          }
          if (kept.size() != 2u * in.c || dflt != in.p0) lookup_rw[k] = {dflt, kept};
          Val h = V(dflt);
          bool all_same = true;
          for (size_t p = 0; p < kept.size(); p += 2) {
            const uint32_t vv = kept[p + 1];
            if (res(vv) != res(dflt)) all_same = false;
            const Val& x = V(vv);
            h.r = rhull(h.r, x.r);
            h.kb = kmeet(h.kb, x.kb);
            if (h.has_set && x.has_set) {
              h.set.insert(h.set.end(), x.set.begin(), x.set.end());
              set_norm(h.set);
            } else {
              h.has_set = false;
              h.set.clear();
            }
          }
          if (all_same) {  // every source is the same value
            alias_to(dflt);
            continue;
          }
          if (W <= 256) r = h;
          break;
        }
        default:
          break;
      }
      tighten(r, W);
      val[d] = std::move(r);
    }
  }
};

}  // namespace

int parse_gen(const Lowered& prog, const uint32_t* blob, size_t n_words, std::vector<GenSpec>& specs,
              std::vector<uint32_t>& consts, std::string& err) {
  if (blob == nullptr || n_words < 4 || blob[0] != MG_GEN_MAGIC) {
    err = "bad generator blob";
    return MG_E_INVALID;
  }
  const uint32_t nc = blob[1], ncw = blob[2];
  if (nc != prog.n_coords || 4ull + 8ull * nc + ncw != n_words) {
    err = "generator does not match program";
    return MG_E_INVALID;
  }
  specs.resize(nc);
  for (uint32_t c = 0; c < nc; c++) std::memcpy(&specs[c], blob + 4 + 8 * c, 32);
  consts.assign(blob + 4 + 8 * nc, blob + n_words);
  for (uint32_t c = 0; c < nc; c++) {
    const GenSpec& s = specs[c];
    const uint32_t L = L_of(prog.coord_width[c]);
    auto in_range = [&](uint64_t off, uint64_t n) { return off + n <= ncw; };
    const uint32_t fix = s.kind >> 8;
    if (fix && !in_range(fix - 1, 2ull * L)) {
      err = "fixed-bit record out of range";
      return MG_E_INVALID;
    }
    switch (s.kind & 0xFFu) {
      case MG_GEN_UNIFORM:
        break;
      case MG_GEN_RANGE:
      case MG_GEN_FIXED:
        if (!in_range(s.p[0], L)) { err = "generator constant out of range"; return MG_E_INVALID; }
        break;
      case MG_GEN_ALIGNED:
        if (!in_range(s.p[0], L) || s.p[1] > 255) { err = "aligned generator"; return MG_E_INVALID; }
        break;
      case MG_GEN_DICT:
      case MG_GEN_MIXED:
        if (s.p[1] == 0 && (s.kind & 0xFFu) == MG_GEN_DICT) { err = "empty dictionary"; return MG_E_INVALID; }
        if (s.p[1] > 65535) { err = "dictionary larger than 65535 entries"; return MG_E_INVALID; }
        if (!in_range(s.p[0], (uint64_t)s.p[1] * L)) { err = "dictionary out of range"; return MG_E_INVALID; }
        if ((s.kind & 0xFFu) == MG_GEN_MIXED) {
          if (s.p[3] != MG_NONE &&
              (s.p[3] >= c || prog.coord_width[s.p[3]] != prog.coord_width[c] ||
               (specs[s.p[3]].kind & 0xFFu) == MG_GEN_LAZY)) {
            err = "copy source must be an earlier, generated coordinate of the same width";
            return MG_E_INVALID;
          }
          if (s.p[6]) {  // clamp record {lo limbs[L], span}: lo + span <= 2^w
            if (!in_range(s.p[6] - 1, (uint64_t)L + 1)) { err = "clamp record out of range"; return MG_E_INVALID; }
            const uint32_t* lo = consts.data() + (s.p[6] - 1);
            const uint64_t span = lo[L] ? lo[L] : (1ull << 32);
            // (lo + span - 1) must fit in w bits
            uint64_t carry = span - 1;
            std::vector<uint32_t> top(L);
            for (uint32_t j = 0; j < L; j++) {
              const uint64_t t = (uint64_t)lo[j] + (carry & 0xFFFFFFFFull);
              top[j] = (uint32_t)t;
              carry = (carry >> 32) + (t >> 32);
            }
            const uint32_t w = prog.coord_width[c];
            const bool over = carry != 0 || ((w & 31u) && (top[L - 1] >> (w & 31u)) != 0);
            if (over) { err = "clamp range exceeds the coordinate width"; return MG_E_INVALID; }
          }
        }
        break;
      case MG_GEN_LAZY:
        break;  // default comes from the program (UFAPP p2); the coordinate is unused
      default:
        err = "unknown generator kind";
        return MG_E_INVALID;
    }
  }
  // longest static COPY chain (the interpreter walks it per candidate)
  std::vector<uint32_t> depth(nc, 0);
  for (uint32_t c = 0; c < nc; c++) {
    const GenSpec& s = specs[c];
    if ((s.kind & 0xFFu) == MG_GEN_MIXED && s.p[3] != MG_NONE) depth[c] = depth[s.p[3]] + 1;
    if (depth[c] > MG_GEN_MAX_COPY_DEPTH) {
      err = "copy chain longer than MG_GEN_MAX_COPY_DEPTH";
      return MG_E_UNSUPPORTED;
    }
  }
  return MG_OK;
}

}  // namespace mg

namespace mg {

// The program a search actually runs once its generator is known.  Every candidate a
// search kernel evaluates is drawn by that generator, so ranges derived from the
// generator specs (clamp records, dictionaries, fixed bits) hold for every lane:
//  * a comparison the ranges decide becomes a literal; an ITE on a literal, a Bool
//    AND/OR with a literal, a LOOKUP with no prior site and a COPY become aliases
//    (their uses are renamed to the value they equal);
//  * an assert decided true disappears; dead instructions are removed;
//  * liveness and slot allocation run again on what is left.
// With specs == nullptr (explicit-coordinate eval) only literal-derived facts are used.
// Verdicts are unchanged for every generated candidate (tests compare the specialised
// interpreter and JIT kernels with the C restatement, which runs the full program).
namespace {

// Keys with literal tails.  LASER addresses a mapping entry as keccak(Concat(key, slot)) with a
// literal slot, so the UF sites' preimages are 512-bit CONCATs whose low 256 bits are literals:
// the site LOOKUPs compare them, the inverse LOOKUPs return them and the injectivity asserts
// compare those with EQ.  A value that is CONCAT(h, T) with a literal T is carried as the pair
// (h, tail id): the id is a small number per distinct literal tail, itself a literal or (through
// a LOOKUP / ITE over values with different tails) a 32-bit value.  Then
//   EQ(x, y)            -> EQ(h_x, h_y), AND EQ(id_x, id_y) unless both ids are literals (equal:
//                          dropped; different: the EQ is the literal false);
//   LOOKUP / ITE values -> narrow twins over the h parts (and over the ids if they differ);
//   LOOKUP keys         -> the h parts, where every key has the same literal tail.
// x:T == y:U iff x == y and T == U, so every verdict is unchanged; the wide CONCATs and LOOKUPs
// die where nothing else reads them.  The interpreter's value file loses half of every such key
// (C2: 112 -> 80 words per lane, so more waves per CU); the JIT half the limbs it selects.
// MYTHGPU_NARROW_TAILS=0: off.  Returns the wide values that got a narrow twin.
std::vector<uint32_t> narrow_literal_tails(std::vector<VInstr>& code, std::vector<uint32_t>& vwidth,
                                           std::vector<uint32_t>& consts, bool& changed) {
  changed = false;
  static const bool on = [] {
    const char* g = getenv("MYTHGPU_NARROW_TAILS");
    return !(g && g[0] == '0');
  }();
  std::vector<uint32_t> twinned;  // wide values that got a narrow twin
  if (!on) return twinned;
  const uint32_t NONE = MG_NONE;
  std::map<uint32_t, std::pair<uint32_t, uint32_t>> lit;  // K_CONST value id -> (width, const offset)
  auto lit_key = [&](uint32_t v) {  // the literal as a string key (width + words), built on demand
    const auto& wo = lit.at(v);
    std::string t = std::to_string(wo.first) + ":";
    for (uint32_t j = 0; j < Lw(wo.first); j++) t += std::to_string(consts.at(wo.second + j)) + ",";
    return t;
  };
  std::map<std::string, uint32_t> tails;  // literal tail -> its id
  std::map<uint32_t, uint32_t> tid_vid;   // tail id -> the value id of its 32-bit literal
  struct Split {
    uint32_t h;
    uint32_t t;     // value id of the tail id (32 bits)
    int64_t tlit;   // the tail id when it is a literal, else -1
  };
  std::map<uint32_t, Split> split;  // value id -> (h, tail id) with value == h:tail
  std::vector<VInstr> outc;
  outc.reserve(code.size() + 8);
  auto fresh = [&](uint32_t w) {
    vwidth.push_back(w);
    return (uint32_t)(vwidth.size() - 1);
  };
  auto literal = [&](uint32_t w, uint32_t word) {  // a new K_CONST of width w <= 32
    const uint32_t v = fresh(w), off = (uint32_t)consts.size();
    consts.push_back(word);
    outc.push_back(VInstr{K_CONST, w, v, NONE, NONE, NONE, off, 0, {}});
    return v;
  };
  auto tid_of = [&](const std::string& t) {
    auto it = tails.find(t);
    const uint32_t id = it != tails.end() ? it->second : (uint32_t)tails.size();
    if (it == tails.end()) tails[t] = id;
    auto iv = tid_vid.find(id);
    if (iv != tid_vid.end()) return Split{NONE, iv->second, (int64_t)id};
    const uint32_t v = literal(32, id);
    tid_vid[id] = v;
    return Split{NONE, v, (int64_t)id};
  };
  auto hw = [&](uint32_t v) { return vwidth[split.at(v).h]; };
  for (VInstr& c : code) {
    if (c.op == K_CONST && c.dst != NONE && c.dst < vwidth.size()) {
      lit[c.dst] = {c.wd, c.p0};
    } else if (c.op == K_CONCAT && c.dst != NONE && lit.count(c.b) && c.a != NONE && c.a < vwidth.size()) {
      const std::string t = lit_key(c.b);
      const Split id = tid_of(t);
      outc.push_back(std::move(c));
      split[outc.back().dst] = Split{outc.back().a, id.t, id.tlit};
      continue;
    } else if (c.op == K_EQ && c.dst != NONE && split.count(c.a) && split.count(c.b) && hw(c.a) == hw(c.b)) {
      const Split x = split[c.a], y = split[c.b];
      changed = true;
      if (x.tlit >= 0 && y.tlit >= 0 && x.tlit != y.tlit) {  // different literal tails: never equal
        const uint32_t off = (uint32_t)consts.size();
        consts.push_back(0u);
        outc.push_back(VInstr{K_CONST, 1, c.dst, NONE, NONE, NONE, off, 0, {}});
        continue;
      }
      c.a = x.h;
      c.b = y.h;
      c.p1 = vwidth[x.h];
      if (!(x.tlit >= 0 && y.tlit >= 0)) {  // computed tail ids: both halves must agree
        const uint32_t eh = fresh(1), et = fresh(1);
        outc.push_back(VInstr{K_EQ, 1, eh, x.h, y.h, NONE, 0, vwidth[x.h], {}});
        outc.push_back(VInstr{K_EQ, 1, et, x.t, y.t, NONE, 0, 32, {}});
        outc.push_back(VInstr{K_AND, 1, c.dst, eh, et, NONE, 0, 1, {}});
        continue;
      }
    } else if (c.op == K_LOOKUP) {
      // keys: the site key and every prior key, all with one literal tail
      bool keys = split.count(c.a) && split[c.a].tlit >= 0;
      for (size_t q = 0; keys && q < c.prior.size(); q += 2)
        keys = split.count(c.prior[q]) && split[c.prior[q]].tlit == split[c.a].tlit && hw(c.prior[q]) == hw(c.a);
      if (keys) {
        changed = true;
        const Split ka = split[c.a];
        for (size_t q = 0; q < c.prior.size(); q += 2) c.prior[q] = split[c.prior[q]].h;
        c.a = ka.h;
        c.b = vwidth[ka.h];
      }
      // values: the default and every prior value
      bool vals = c.dst != NONE && split.count(c.p0);
      bool one_tail = vals;
      for (size_t q = 1; vals && q < c.prior.size(); q += 2) {
        vals = split.count(c.prior[q]) && hw(c.prior[q]) == hw(c.p0);
        one_tail = one_tail && vals && split[c.prior[q]].tlit >= 0 && split[c.prior[q]].tlit == split[c.p0].tlit;
      }
      one_tail = one_tail && split[c.p0].tlit >= 0;
      if (vals) {
        const Split d0 = split[c.p0];
        VInstr n = c;
        n.dst = fresh(vwidth[d0.h]);
        n.wd = vwidth[d0.h];
        n.p0 = d0.h;
        for (size_t q = 1; q < n.prior.size(); q += 2) n.prior[q] = split[n.prior[q]].h;
        Split r{n.dst, d0.t, d0.tlit};
        outc.push_back(c);
        outc.push_back(std::move(n));
        if (!one_tail) {
          VInstr t = c;
          t.dst = fresh(32);
          t.wd = 32;
          t.p0 = d0.t;
          for (size_t q = 1; q < t.prior.size(); q += 2) t.prior[q] = split[t.prior[q]].t;
          r.t = t.dst;
          r.tlit = -1;
          outc.push_back(std::move(t));
        }
        split[c.dst] = r;
        twinned.push_back(c.dst);
        continue;
      }
    } else if (c.op == K_ITE && c.dst != NONE && split.count(c.b) && split.count(c.c) && hw(c.b) == hw(c.c)) {
      const Split x = split[c.b], y = split[c.c];
      VInstr n = c;
      n.dst = fresh(vwidth[x.h]);
      n.wd = vwidth[x.h];
      n.b = x.h;
      n.c = y.h;
      Split r{n.dst, x.t, x.tlit};
      outc.push_back(c);
      outc.push_back(std::move(n));
      if (!(x.tlit >= 0 && x.tlit == y.tlit)) {
        VInstr t = c;
        t.dst = fresh(32);
        t.wd = 32;
        t.b = x.t;
        t.c = y.t;
        r.t = t.dst;
        r.tlit = -1;
        outc.push_back(std::move(t));
      }
      split[c.dst] = r;
      twinned.push_back(c.dst);
      continue;
    }
    outc.push_back(std::move(c));
  }
  code.swap(outc);
  changed = changed || !twinned.empty();
  return twinned;
}

}  // namespace

// A search program's constraints, heavy ones last (the interpreter's and the O3 kernel's order; the
// first tier orders its own the same way, jit_asm.cpp heavy_last_roots).  Each ASSERT is emitted
// right after the cone it needs, so a wave that leaves at the first ASSERT all its lanes failed skips
// every later cone.  A constraint whose not-yet-emitted cone holds Keccak, EXP or a division goes
// after the light ones (which keep program order); the heavy ones follow cheapest remaining cone
// first.  A program without such an operator is returned unchanged.  MYTHGPU_HEAVY_LAST=0: off.
static void heavy_last(std::vector<VInstr>& list) {
  static const bool on = [] {
    const char* g = getenv("MYTHGPU_HEAVY_LAST");
    return !(g && g[0] == '0');
  }();
  auto heavy = [](uint32_t op) {
    return op == K_KECCAK || op == K_EXP || op == K_UDIV || op == K_UREM || op == K_SDIV || op == K_SREM || op == K_SMOD;
  };
  if (!on || std::none_of(list.begin(), list.end(), [&](const VInstr& c) { return heavy(c.op); })) return;
  // rough VALU per candidate on the compiled kernels (the first tier's op_weight): which heavy cone is
  // cheapest (a Keccak-f[1600] ~2,500, EXP ~1,500, a division ~600)
  auto weight = [](const VInstr& in) -> uint64_t {
    const uint64_t L = std::max<uint32_t>(1, Lw(std::max(in.wd, in.op >= K_EQ && in.op <= K_UMUL_NOOVF ? in.p1 : in.wd)));
    switch (in.op) {
      case K_KECCAK: return 2500ull * (in.p0 / 136u + 1u);
      case K_EXP: return 1500;
      case K_UDIV: case K_UREM: case K_SDIV: case K_SREM: case K_SMOD: return 600;
      case K_MUL: return 4 * L * L;
      case K_UMUL_NOOVF: return 8 * L * L;
      case K_SHL: case K_LSHR: case K_ASHR: return 4 * L;
      case K_LOOKUP: return 2ull * Lw(in.b) * std::max<uint32_t>(1, in.c);
      case K_COORD: return 8 * L;
      default: return L;
    }
  };
  std::map<uint32_t, int32_t> def;
  for (size_t k = 0; k < list.size(); k++)
    if (list[k].dst != MG_NONE && !def.count(list[k].dst)) def[list[k].dst] = (int32_t)k;
  auto operands = [&](const VInstr& c, std::vector<int32_t>& out) {
    out.clear();
    auto add = [&](uint32_t x) {
      auto it = x == MG_NONE ? def.end() : def.find(x);
      if (it != def.end()) out.push_back(it->second);
    };
    if (c.op == K_LOOKUP) {
      add(c.a);
      add(c.p0);
      for (uint32_t x : c.prior) add(x);
    } else if (c.op == K_CONCAT || c.op == K_EXTRACT || c.op == K_ZEXT || c.op == K_SEXT || c.op == K_KECCAK ||
               c.op == K_ASSERT || c.op == K_WATCH || c.op == K_COPY) {
      add(c.a);
      add(c.b);
    } else if (c.op != K_CONST && c.op != K_COORD) {
      add(c.a);
      add(c.b);
      add(c.c);
    }
  };
  std::vector<char> done(list.size(), 0);
  std::vector<int32_t> order, ops, st, mark(list.size(), -1);
  int32_t stamp = 0;
  auto visit = [&](int32_t root) {  // operands first, depth-first
    std::vector<std::pair<int32_t, std::vector<int32_t>>> stk;
    stk.push_back({root, {}});
    operands(list[root], stk.back().second);
    std::reverse(stk.back().second.begin(), stk.back().second.end());
    while (!stk.empty()) {
      auto& top = stk.back();
      if (done[top.first]) {
        stk.pop_back();
        continue;
      }
      if (!top.second.empty()) {
        const int32_t o = top.second.back();
        top.second.pop_back();
        if (!done[o]) {
          stk.push_back({o, {}});
          operands(list[o], stk.back().second);
          std::reverse(stk.back().second.begin(), stk.back().second.end());
        }
        continue;
      }
      done[top.first] = 1;
      order.push_back(top.first);
      stk.pop_back();
    }
  };
  auto cone = [&](int32_t r, bool& hv) -> uint64_t {
    uint64_t c = 0;
    hv = false;
    st.assign(1, r);
    mark[r] = ++stamp;
    while (!st.empty()) {
      const int32_t x = st.back();
      st.pop_back();
      const VInstr& in = list[x];
      c += weight(in);
      hv = hv || heavy(in.op);
      operands(in, ops);
      for (int32_t o : ops)
        if (!done[o] && mark[o] != stamp) {
          mark[o] = stamp;
          st.push_back(o);
        }
    }
    return c;
  };
  std::vector<int32_t> roots;
  for (size_t k = 0; k < list.size(); k++)
    if (list[k].op == K_ASSERT || list[k].op == K_WATCH) roots.push_back((int32_t)k);
  std::vector<char> taken(roots.size(), 0);
  for (size_t step = 0; step < roots.size(); step++) {
    size_t pick = roots.size();
    uint64_t best = UINT64_MAX;
    for (size_t i = 0; i < roots.size(); i++) {
      if (taken[i]) continue;
      bool hv = false;
      const uint64_t c = cone(roots[i], hv);
      if (!hv) {
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
  for (size_t k = 0; k < list.size(); k++)
    if (!done[k]) visit((int32_t)k);
  std::vector<VInstr> out;
  out.reserve(list.size());
  for (int32_t k : order) out.push_back(std::move(list[k]));
  list.swap(out);
}

int specialize_program(const Lowered& in, const std::vector<GenSpec>* specs, const std::vector<uint32_t>* gconsts,
                       Lowered& out, std::string& err, bool keep_watch, bool keep_asserts) {
  try {
    const uint32_t NONE = MG_NONE;
    Analysis A(in, specs, gconsts);
    A.analyze(specs != nullptr);
    const size_t nv = in.vwidth.size();
    out = in;
    out.code.clear();
    out.aux.clear();
    std::vector<uint32_t> vwidth = in.vwidth;
    // rewritten SSA list (value ids are kept; aliases renamed to their representative)
    std::vector<VInstr> code;
    code.reserve(in.vcode.size());
    for (size_t k = 0; k < in.vcode.size(); k++) {
      const Instr& c = in.vcode[k];
      if (A.skip[k]) continue;
      auto R = [&](uint32_t v) { return v == NONE || v >= nv ? v : A.res(v); };
      if (c.dst != NONE && c.dst < nv && A.fold[c.dst] >= 0 && c.op != K_CONST && c.op != K_COORD) {
        const uint32_t off = (uint32_t)out.consts.size();
        out.consts.push_back((uint32_t)A.fold[c.dst]);
        code.push_back(VInstr{K_CONST, 1, c.dst, NONE, NONE, NONE, off, 0, {}});
        continue;
      }
      {  // a value every candidate gives the same (e.g. the low bits of an aligned site) is a literal
        U256 x;
        if (c.dst != NONE && c.dst < nv && c.wd <= 256 && c.op != K_CONST && c.op != K_COORD &&
            c.op != K_ASSERT && c.op != K_WATCH && Analysis::exact_of(A.val[c.dst], &x)) {
          const uint32_t off = (uint32_t)out.consts.size();
          for (uint32_t j = 0; j < Lw(c.wd); j++) out.consts.push_back((uint32_t)(x.w[j / 2] >> (32 * (j % 2))));
          code.push_back(VInstr{K_CONST, c.wd, c.dst, NONE, NONE, NONE, off, 0, {}});
          continue;
        }
      }
      if ((c.op == K_EXTRACT || c.op == K_CONCAT) && c.dst < nv && A.psrc[c.dst] != NONE) {
        const uint32_t src = A.psrc[c.dst];
        code.push_back(VInstr{K_EXTRACT, c.wd, c.dst, src, NONE, NONE, A.plo[c.dst], in.vwidth[src], {}});
        continue;
      }
      auto rw = A.rewrite.find(k);
      if (rw != A.rewrite.end()) {
        const Instr& x = rw->second;
        code.push_back(VInstr{x.op, x.wd, x.dst, R(x.a), R(x.b), R(x.c), x.p0, x.p1, {}});
        continue;
      }
      VInstr v{c.op, c.wd, c.dst, R(c.a), R(c.b), R(c.c), c.p0, c.p1, {}};
      if (c.op == K_LOOKUP) {
        v.a = R(c.a);
        v.b = c.b;  // key width
        v.c = c.c;  // number of priors
        v.p0 = R(c.p0);
        auto lr = A.lookup_rw.find(k);
        if (lr != A.lookup_rw.end()) {
          v.p0 = R(lr->second.first);
          v.c = (uint32_t)(lr->second.second.size() / 2);
          for (uint32_t x : lr->second.second) v.prior.push_back(R(x));
        } else {
          for (uint32_t p = 0; p < c.c; p++) {
            v.prior.push_back(R(in.vaux[c.p1 + 2 * p]));
            v.prior.push_back(R(in.vaux[c.p1 + 2 * p + 1]));
          }
        }
      } else if (c.op == K_CONST || c.op == K_COORD) {
        v.a = v.b = v.c = NONE;
      }
      code.push_back(std::move(v));
    }
    std::vector<VInstr> wide = code;
    bool narrowed = false;
    (void)narrow_literal_tails(code, vwidth, out.consts, narrowed);
    const size_t nw = vwidth.size();  // with the narrow twins' values
    // dead code: keep asserts (unless dropped: the model read-back of a known hit), watches
    // and whatever they transitively use
    auto dce = [&](std::vector<VInstr>& list) {
      const size_t nw = vwidth.size();  // the rewrites below add values
      std::vector<char> live(nw, 0), keep(list.size(), 0);
      for (size_t k = list.size(); k-- > 0;) {
        const VInstr& c = list[k];
        const bool side = (c.op == K_ASSERT && keep_asserts) || (c.op == K_WATCH && keep_watch);
        if (!side && (c.dst == NONE || c.dst >= nw || !live[c.dst])) continue;
        keep[k] = 1;
        auto use = [&](uint32_t x) {
          if (x != NONE && x < nw) live[x] = 1;
        };
        if (c.op == K_LOOKUP) {
          use(c.a);
          use(c.p0);
          for (uint32_t x : c.prior) use(x);
        } else if (c.op == K_CONCAT || c.op == K_EXTRACT || c.op == K_ZEXT || c.op == K_SEXT || c.op == K_KECCAK ||
                   c.op == K_ASSERT || c.op == K_WATCH || c.op == K_COPY) {
          use(c.a);
          use(c.b);
        } else if (c.op != K_CONST && c.op != K_COORD) {
          use(c.a);
          use(c.b);
          use(c.c);
        }
      }
      std::vector<VInstr> kept;
      kept.reserve(list.size());
      for (size_t k = 0; k < list.size(); k++)
        if (keep[k] && (keep_watch || list[k].op != K_WATCH)) kept.push_back(std::move(list[k]));
      return kept;
    };
    std::vector<VInstr> kept = dce(code);
    // the JIT keeps the wide program: it folds literal limbs by itself, and a wide value that stays
    // live next to its narrow twin (a LOOKUP over keys with different tails still reads it: C4) is
    // extra work there; measured on the compiled kernels: C2 -1.9 %, C4 +0.4 % narrowed
    const uint64_t ops = in.limb_ops;  // algorithmic work is the query's, not what survives
    out.limb_ops = 0;
    // the compiled kernels' list also takes the lookup-compare pushdown; the interpreter's slot code
    // does not (each pushed compare is one more dispatch there)
    bool pushed = false, pruned = false, folded = false;
    // MYTHGPU_FOLD_NOT=0: keep NOT(compare) as two instructions (diagnostic)
    static const bool fold_on = [] {
      const char* g = getenv("MYTHGPU_FOLD_NOT");
      return !(g && g[0] == '0');
    }();
    auto fold_nots = [&] { return fold_on; };
    auto jit_rewrites = [&](const std::vector<VInstr>& list) {
      std::vector<VInstr> r = prune_guarded_lookups(list, vwidth.size(), &pruned);
      if (pruned) r = dce(r);
      // to a fixed point (bounded): a pushed compare of a lookup whose values are lookups in turn —
      // LASER's nested keccak inverse maps (C4: the preimage of one hash compared with the preimage
      // of another) — is pushed again, so the inner 512-bit select chains go too
      for (int round = 0; round < 4; round++) {
        bool again = false;
        r = push_eq_into_lookup(r, vwidth, out.consts, &again);
        if (!again) break;
        pushed = true;
        r = dce(r);
      }
      if (fold_nots()) r = fold_not_compares(r, vwidth.size(), &folded);
      return r;
    };
    // a search program (a generator: early exit) with heavy operators: heavy constraints last
    const bool order = specs != nullptr;
    if (order) heavy_last(kept);
    if (narrowed) {
      std::vector<VInstr> kept_wide = jit_rewrites(dce(wide));
      if (order) heavy_last(kept_wide);
      allocate(kept_wide, vwidth, out, &kept);
    } else {
      std::vector<VInstr> jit_list = jit_rewrites(kept);
      if (order) heavy_last(jit_list);
      if (pushed || pruned || folded)
        allocate(jit_list, vwidth, out, &kept);
      else
        allocate(kept, vwidth, out);
    }
    out.limb_ops = ops;
    return MG_OK;
  } catch (const Fail& f) {
    err = f.msg;
    return f.code;
  } catch (const std::exception& e) {
    err = e.what();
    return MG_E_INVALID;
  }
}

}  // namespace mg
