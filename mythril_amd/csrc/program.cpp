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
#include <map>
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
void allocate(const std::vector<VInstr>& code, const std::vector<uint32_t>& vwidth, Lowered& out) {
  const uint32_t NONE = MG_NONE;
  const size_t nv = vwidth.size();
  out.vcode.clear();
  out.vaux.clear();
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
  std::vector<uint32_t> slot(nv, NONE);
  std::vector<std::vector<uint32_t>> dies(code.size());
  for (size_t v = 0; v < nv; v++) {
    if (def[v] < 0) continue;
    int64_t d = std::max(last[v], def[v]);
    dies[(size_t)d].push_back((uint32_t)v);
  }
  Alloc al;
  uint32_t dbg_high = 0;
  out.code.clear();
  out.aux.clear();
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
      in.p1 = (uint32_t)out.aux.size();
      for (uint32_t v : c.prior) out.aux.push_back(S(v));
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
    out.code.push_back(in);
    {
      Instr vi{c.op, c.wd, c.dst, c.a, c.b, c.c, c.p0, c.p1};
      if (c.op == K_LOOKUP) {
        vi.p1 = (uint32_t)out.vaux.size();
        for (uint32_t v : c.prior) out.vaux.push_back(v);
      }
      out.vcode.push_back(vi);
    }
    // cost
    uint32_t wa = c.p1;
    if (c.op == K_LOOKUP) {
      out.limb_ops += 3ull * L_of(c.b) * c.c + L_of(c.wd);
    } else if (c.op == K_KECCAK) {
      out.limb_ops += 7500ull * (c.p0 / 136 + 1);
    } else {
      out.limb_ops += op_cost(c.op, c.wd, wa ? wa : c.wd);
    }
    for (uint32_t v : dies[k]) al.release(slot[v], L_of(vwidth[v]));
    if (getenv("MYTHGPU_DEBUG_ALLOC") && al.high() > dbg_high) {
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
  out.value_words = std::max<uint32_t>(al.high(), 1);
  out.vwidth = vwidth;
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

    allocate(code, vwidth, out);
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

struct Analysis {
  const Lowered& P;
  const std::vector<GenSpec>* specs;
  const std::vector<uint32_t>* gconsts;
  Analysis(const Lowered& p, const std::vector<GenSpec>* s, const std::vector<uint32_t>* g) : P(p), specs(s), gconsts(g) {}
  // rng[id]: when known, the value lies in [lo, hi] (so it fits in 64 bits).  In the
  // search kernel a coordinate's range comes from its generator spec, which bounds
  // EVERY candidate the kernel evaluates (clamp records, dictionaries, fixed bits), so a
  // comparison decided by the ranges is decided for every candidate: it folds to a
  // literal, an ITE on it becomes an alias of the chosen arm, and bits() then looks
  // through it (e.g. the calldata guard If(k < size, calldata[k], 0) with size drawn
  // from [68, 2^32) collapses to the byte, and a CALLDATALOAD to its AUX word).
  struct Rng {
    bool k = false;
    uint64_t lo = 0, hi = 0;
  };
  std::vector<Rng> rng;
  // psrc/plo: the value is bits [plo, plo + width) of value psrc (a chain of EXTRACTs, and
  // CONCATs of adjacent slices of one value, e.g. a CALLDATALOAD of an AUX word's bytes)
  std::vector<uint32_t> psrc, plo;
  std::vector<int8_t> fold;       // per id: -1, or the folded Bool value
  std::vector<uint32_t> alias;    // per id: the id it equals (itself if none)
  std::vector<char> skip;         // per instruction: defines an alias / a decided assert
  std::vector<Rng> crng;          // per coordinate (search mode)

  uint32_t res(uint32_t id) const {
    if (alias.empty() || id >= alias.size()) return id;
    while (alias[id] != id) id = alias[id];
    return id;
  }
  static Rng full(uint32_t w) {
    Rng r;
    if (w <= 64) {
      r.k = true;
      r.hi = w == 64 ? ~0ull : ((1ull << w) - 1ull);
    }
    return r;
  }
  static Rng exact(uint64_t v) {
    Rng r;
    r.k = true;
    r.lo = r.hi = v;
    return r;
  }
  static Rng hull(const Rng& a, const Rng& b) {
    Rng r;
    if (!a.k || !b.k) return r;
    r.k = true;
    r.lo = std::min(a.lo, b.lo);
    r.hi = std::max(a.hi, b.hi);
    return r;
  }
  // limbs [0, L) as one u64 if every limb >= 2 is zero
  static bool fits64(const uint32_t* x, uint32_t L, uint64_t* v) {
    for (uint32_t j = 2; j < L; j++)
      if (x[j]) return false;
    *v = (uint64_t)x[0] | (L > 1 ? (uint64_t)x[1] << 32 : 0ull);
    return true;
  }

  // range of a generated coordinate's final value (include/mythgpu.h GEN3)
  Rng coord_range(uint32_t c) const {
    const GenSpec& sp = (*specs)[c];
    const uint32_t w = P.coord_width[c], L = Lw(w), kind = sp.kind & 0xFFu;
    const auto& G = *gconsts;
    const unsigned __int128 wlim = w >= 128 ? ~(unsigned __int128)0 : (((unsigned __int128)1 << w) - 1);
    Rng r;
    switch (kind) {
      case MG_GEN_FIXED: {
        uint64_t v;
        if (fits64(&G[sp.p[0]], L, &v)) r = exact(v);
        break;
      }
      case MG_GEN_DICT:
      case MG_GEN_MIXED: {
        Rng d;  // dictionary hull
        bool ok = sp.p[1] > 0;
        for (uint32_t e = 0; ok && e < sp.p[1]; e++) {
          uint64_t v;
          if (!fits64(&G[sp.p[0] + e * L], L, &v)) ok = false;
          else d = d.k ? hull(d, exact(v)) : exact(v);
        }
        if (kind == MG_GEN_DICT) {
          if (ok) r = d;
          break;
        }
        if (sp.p[6]) {  // clamp record: the final value is inside [lo, lo + span)
          uint64_t lo;
          const uint32_t rec = sp.p[6] - 1;
          if (fits64(&G[rec], L, &lo)) {
            const uint64_t span = G[rec + L] ? G[rec + L] : (1ull << 32);
            if ((unsigned __int128)lo + span - 1 <= (unsigned __int128)~0ull) {
              r.k = true;
              r.lo = lo;
              r.hi = lo + span - 1;
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
          else u = have ? hull(u, x) : x;
          have = true;
        };
        Rng cd;  // COPY / DICT part, before the delta
        bool cd_have = false, cd_unknown = false;
        if (pc) {
          const Rng s = crng[sp.p[3]];
          if (!s.k) cd_unknown = true;
          else cd = s;
          cd_have = true;
        }
        if (pd) {
          if (!ok) cd_unknown = true;
          else cd = cd_have && cd.k ? hull(cd, d) : d;
          cd_have = true;
        }
        if (cd_have) {
          if (cd_unknown) add(Rng{});
          else if (sp.p[5]) {  // +/-2 at most, no wrap
            if (cd.lo >= 2 && (unsigned __int128)cd.hi + 2 <= wlim && cd.hi + 2 > cd.hi) {
              Rng x;
              x.k = true;
              x.lo = cd.lo - 2;
              x.hi = cd.hi + 2;
              add(x);
            } else {
              add(full(w));
            }
          } else {
            add(cd);
          }
        }
        const uint32_t sb = std::min(w, sp.p[4] >> 16);
        if (ps) add(full(sb));
        if (pc + pd + ps < 65536u) add(full(w));
        if (have && !unknown) r = u;
        break;
      }
      case MG_GEN_RANGE: {
        uint64_t lo;
        if (fits64(&G[sp.p[0]], L, &lo)) {
          const uint64_t span = sp.p[1] ? sp.p[1] : (1ull << 32);
          if ((unsigned __int128)lo + span - 1 <= wlim && (unsigned __int128)lo + span - 1 <= (unsigned __int128)~0ull) {
            r.k = true;
            r.lo = lo;
            r.hi = lo + span - 1;
          }
        }
        break;
      }
      case MG_GEN_ALIGNED: {
        uint64_t lo;
        if (fits64(&G[sp.p[0]], L, &lo) && sp.p[1] < 64) {
          const unsigned __int128 cnt = sp.p[2] ? sp.p[2] : (1ull << 32);
          const unsigned __int128 top = (unsigned __int128)lo + ((cnt - 1) << sp.p[1]);
          if (top <= wlim && top <= (unsigned __int128)~0ull) {
            r.k = true;
            r.lo = lo;
            r.hi = (uint64_t)top;
          }
        }
        break;
      }
      default:  // UNIFORM / LAZY
        r = full(w);
        break;
    }
    if (!r.k) r = full(w);
    if (const uint32_t fix = sp.kind >> 8) {  // (v & ~m) | val lies in [val, val | ~m]
      const uint32_t f = fix - 1;
      uint64_t m, val;
      std::vector<uint32_t> nm(L);
      for (uint32_t j = 0; j < L; j++) nm[j] = ~G[f + j];
      if (w & 31) nm[L - 1] &= (1u << (w & 31)) - 1u;
      if (fits64(&G[f + L], L, &val) && fits64(nm.data(), L, &m)) {
        r.k = true;
        r.lo = val;
        r.hi = val | m;
      } else {
        r = Rng{};
      }
    }
    return r;
  }

  // decide a comparison from operand ranges: -1 undecided, else 0 / 1
  static int decide(uint32_t op, const Rng& a, const Rng& b, uint32_t wa) {
    if (!a.k || !b.k) return -1;
    if (op == K_SLT || op == K_SLE) {
      const uint64_t sign = wa >= 65 ? 0ull : (1ull << (wa - 1));
      if (sign && (a.hi >= sign || b.hi >= sign)) return -1;  // a negative value may be inside
      op = op == K_SLT ? K_ULT : K_ULE;
    }
    switch (op) {
      case K_ULT:
        if (a.hi < b.lo) return 1;
        if (a.lo >= b.hi) return 0;
        return -1;
      case K_ULE:
        if (a.hi <= b.lo) return 1;
        if (a.lo > b.hi) return 0;
        return -1;
      case K_EQ:
        if (a.lo == a.hi && b.lo == b.hi && a.lo == b.lo) return 1;
        if (a.hi < b.lo || b.hi < a.lo) return 0;
        return -1;
      default:
        return -1;
    }
  }

  void analyze(bool search) {
    const size_t nv = P.vwidth.size();
    rng.assign(nv, Rng{});
    psrc.assign(nv, MG_NONE);
    plo.assign(nv, 0);
    fold.assign(nv, -1);
    alias.resize(nv);
    for (size_t i = 0; i < nv; i++) alias[i] = (uint32_t)i;
    skip.assign(P.vcode.size(), 0);
    if (search && specs) {
      crng.assign(P.n_coords, Rng{});
      for (uint32_t c = 0; c < P.n_coords; c++) crng[c] = coord_range(c);
    }
    for (size_t k = 0; k < P.vcode.size(); k++) {
      const Instr& in = P.vcode[k];
      const uint32_t d = in.dst, W = in.wd;
      auto R = [&](uint32_t id) { return rng[res(id)]; };
      auto F = [&](uint32_t id) { return (int)fold[res(id)]; };
      auto alias_to = [&](uint32_t src) {
        alias[d] = res(src);
        rng[d] = rng[res(src)];
        fold[d] = fold[res(src)];
        skip[k] = 1;
      };
      auto set_fold = [&](int v) {
        fold[d] = (int8_t)v;
        rng[d] = exact((uint64_t)v);
      };
      if (d == MG_NONE || d >= nv) {
        if (in.op == K_ASSERT && F(in.a) == 1) skip[k] = 1;
        continue;
      }
      Rng r = full(W);
      switch (in.op) {
        case K_CONST: {
          uint64_t v;
          if (fits64(&P.consts[in.p0], Lw(W), &v)) r = exact(v);
          break;
        }
        case K_COORD:
          if (search && specs) r = crng[in.p0];
          break;
        case K_COPY:
          alias_to(in.a);
          continue;
        case K_ZEXT:
          if (R(in.a).k) r = R(in.a);
          break;
        case K_EXTRACT: {
          const Rng a = R(in.a);
          if (a.k && in.p0 < 64 && (W >= 64 || (a.hi >> in.p0) < (1ull << W))) {
            r.k = true;
            r.lo = a.lo >> in.p0;
            r.hi = a.hi >> in.p0;
          } else if (a.k && in.p0 >= 64) {
            r = exact(0);
          }
          const uint32_t ra = res(in.a);
          const uint32_t src = psrc[ra] != MG_NONE ? psrc[ra] : ra;
          const uint32_t lo = (psrc[ra] != MG_NONE ? plo[ra] : 0u) + in.p0;
          if (lo == 0 && W == P.vwidth[src]) {
            alias_to(src);
            continue;
          }
          psrc[d] = src;
          plo[d] = lo;
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
              r = full(W);
              break;
            }
          }
          const Rng a = R(in.a), b = R(in.b);
          const uint32_t wb = in.p1;
          if (a.k && b.k && wb < 64 && (a.hi >> (64 - wb)) == 0) {
            r.k = true;
            r.lo = (a.lo << wb) | b.lo;
            r.hi = (a.hi << wb) | b.hi;
          }
          break;
        }
        case K_AND:
        case K_OR:
        case K_XOR: {
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
            break;
          }
          const Rng a = R(in.a), b = R(in.b);
          if (in.op == K_AND) {
            if (a.k || b.k) {
              r.k = true;
              r.lo = 0;
              r.hi = std::min(a.k ? a.hi : ~0ull, b.k ? b.hi : ~0ull);
            }
          } else if (a.k && b.k) {
            const uint64_t m = std::max(a.hi, b.hi);
            r.k = true;
            r.lo = 0;
            r.hi = m ? (~0ull >> __builtin_clzll(m)) : 0ull;
          }
          break;
        }
        case K_NOT:
          if (W == 1 && F(in.a) >= 0) {
            set_fold(1 - F(in.a));
            continue;
          }
          break;
        case K_ITE: {
          const int fc = F(in.a);
          if (fc >= 0) {
            alias_to(fc ? in.b : in.c);
            continue;
          }
          const Rng h = hull(R(in.b), R(in.c));
          if (h.k) r = h;
          break;
        }
        case K_ADD: {
          const Rng a = R(in.a), b = R(in.b);
          if (a.k && b.k && (unsigned __int128)a.hi + b.hi <= (unsigned __int128)full(std::min(W, 64u)).hi) {
            r.k = true;
            r.lo = a.lo + b.lo;
            r.hi = a.hi + b.hi;
          }
          break;
        }
        case K_SUB: {
          const Rng a = R(in.a), b = R(in.b);
          if (a.k && b.k && a.lo >= b.hi) {
            r.k = true;
            r.lo = a.lo - b.hi;
            r.hi = a.hi - b.lo;
          }
          break;
        }
        case K_EQ:
        case K_ULT:
        case K_ULE:
        case K_SLT:
        case K_SLE: {
          const int v = decide(in.op, R(in.a), R(in.b), in.p1);
          if (v >= 0) {
            set_fold(v);
            continue;
          }
          break;
        }
        case K_LOOKUP: {
          if (in.c == 0) {  // no earlier site can share the key: the default
            alias_to(in.p0);
            continue;
          }
          Rng h = R(in.p0);
          for (uint32_t p = 0; p < in.c && h.k; p++) h = hull(h, R(P.vaux[in.p1 + 2 * p + 1]));
          if (h.k) r = h;
          break;
        }
        default:
          break;
      }
      if (r.k && W < 64) {  // intersect with the width
        const uint64_t m = (1ull << W) - 1ull;
        if (r.hi > m) r = full(W);
      }
      rng[d] = r;
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
      if ((c.op == K_EXTRACT || c.op == K_CONCAT) && c.dst < nv && A.psrc[c.dst] != NONE) {
        const uint32_t src = A.psrc[c.dst];
        code.push_back(VInstr{K_EXTRACT, c.wd, c.dst, src, NONE, NONE, A.plo[c.dst], in.vwidth[src], {}});
        continue;
      }
      VInstr v{c.op, c.wd, c.dst, R(c.a), R(c.b), R(c.c), c.p0, c.p1, {}};
      if (c.op == K_LOOKUP) {
        v.a = R(c.a);
        v.b = c.b;  // key width
        v.c = c.c;  // number of priors
        v.p0 = R(c.p0);
        for (uint32_t p = 0; p < c.c; p++) {
          v.prior.push_back(R(in.vaux[c.p1 + 2 * p]));
          v.prior.push_back(R(in.vaux[c.p1 + 2 * p + 1]));
        }
      } else if (c.op == K_CONST || c.op == K_COORD) {
        v.a = v.b = v.c = NONE;
      }
      code.push_back(std::move(v));
    }
    // dead code: keep asserts (unless dropped: the model read-back of a known hit), watches
    // and whatever they transitively use
    std::vector<char> live(nv, 0), keep(code.size(), 0);
    for (size_t k = code.size(); k-- > 0;) {
      const VInstr& c = code[k];
      const bool side = (c.op == K_ASSERT && keep_asserts) || (c.op == K_WATCH && keep_watch);
      if (!side && (c.dst == NONE || c.dst >= nv || !live[c.dst])) continue;
      keep[k] = 1;
      auto use = [&](uint32_t x) {
        if (x != NONE && x < nv) live[x] = 1;
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
    kept.reserve(code.size());
    for (size_t k = 0; k < code.size(); k++)
      if (keep[k] && (keep_watch || code[k].op != K_WATCH)) kept.push_back(std::move(code[k]));
    const uint64_t ops = in.limb_ops;  // algorithmic work is the query's, not what survives
    out.limb_ops = 0;
    allocate(kept, vwidth, out);
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
