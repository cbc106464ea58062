/*
 * ORACLE (test infrastructure only) — plain-C restatement of z3's
 * model.eval for LASER's term vocabulary, driven by the engine's program v1
 * format, plus a restatement of the engine's candidate generator so that it
 * evaluates EXACTLY the candidates the GPU evaluates.
 *
 * Used by tests/ (hit counts / first hit must equal the GPU's) and by
 * bench.py's cpu_baseline leg ("port": timed on the host cores with OpenMP).
 * Never linked into the product.  Semantics restated (SMT-LIB QF_ABV, what z3
 * evaluates for mythril/laser/smt terms):
 *   bvudiv x 0 = ~0, bvurem x 0 = x, bvsdiv/bvsrem/bvsmod by the msb case
 *   split, shifts >= w saturate, bvumul_noovfl = product fits in w bits;
 *   arrays/UFs under a finite model with per-candidate first-occurrence
 *   tables (the model the GPU reads back, mythril_amd/ssa.py model_from_sites).
 * Independent code: 64-bit limbs (the GPU uses 32-bit limbs), recursive
 * descent over nodes, no shared source with mythril_amd/csrc.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAXW 16 /* 64-bit words per value: 1024 bits */
#define NONE 0xFFFFFFFFu

typedef struct { uint64_t w[MAXW]; } val_t;

typedef struct {
  uint32_t op, width, a, b, c, p0, p1, p2;
} node_t;

enum {
  OP_CONST = 0, OP_VAR, OP_ADD, OP_SUB, OP_MUL, OP_UDIV, OP_UREM, OP_SDIV, OP_SREM, OP_SMOD, OP_AND, OP_OR,
  OP_XOR, OP_NOT, OP_NEG, OP_SHL, OP_LSHR, OP_ASHR, OP_CONCAT, OP_EXTRACT, OP_ZEXT, OP_SEXT, OP_ITE, OP_EQ,
  OP_ULT, OP_ULE, OP_SLT, OP_SLE, OP_UMUL_NOOVF, OP_ARR_VAR, OP_ARR_K, OP_ARR_STORE, OP_SELECT, OP_UFAPP,
  OP_KECCAK, OP_EXP
};

typedef struct {
  uint32_t n_nodes, n_roots, n_coords, n_tables, n_consts;
  const node_t* nodes;
  const uint32_t* roots;
  const uint32_t* coords; /* 4 words each */
  const uint32_t* tables;
  const uint32_t* consts;
  /* generator */
  uint32_t gen_n;
  const uint32_t* specs; /* 8 words each */
  const uint32_t* gconsts;
} prog_t;

static int nw(uint32_t width) { return (int)((width + 63) / 64); }

static void vzero(val_t* v) { memset(v, 0, sizeof(*v)); }

static void vmask(val_t* v, uint32_t width) {
  int n = nw(width);
  for (int i = n; i < MAXW; i++) v->w[i] = 0;
  uint32_t r = width % 64;
  if (r) v->w[n - 1] &= (1ull << r) - 1;
}

static int vbit(const val_t* v, uint32_t i) { return (int)((v->w[i / 64] >> (i % 64)) & 1); }

static int veq(const val_t* a, const val_t* b) { return memcmp(a, b, sizeof(*a)) == 0; }

static int vult(const val_t* a, const val_t* b) {
  for (int i = MAXW - 1; i >= 0; i--)
    if (a->w[i] != b->w[i]) return a->w[i] < b->w[i];
  return 0;
}

static int viszero(const val_t* a) {
  for (int i = 0; i < MAXW; i++)
    if (a->w[i]) return 0;
  return 1;
}

/* Keccak-256 (0x01 padding, rate 136), FIPS-202 Keccak-f[1600] on 64-bit lanes,
 * as _pysha3 / ethereum.utils.sha3 (keccak_function_manager.py:44-57).  Pinned by
 * the KATs in tests/golden/keccak_kat.json through tests/test_cport.py. */
static const uint64_t KRC[24] = {
  0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808Aull, 0x8000000080008000ull,
  0x000000000000808Bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
  0x000000000000008Aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000Aull,
  0x000000008000808Bull, 0x800000000000008Bull, 0x8000000000008089ull, 0x8000000000008003ull,
  0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800Aull, 0x800000008000000Aull,
  0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};

static uint64_t rotl64(uint64_t x, unsigned r) { return r ? (x << r) | (x >> (64 - r)) : x; }

static void keccak_f1600(uint64_t a[25]) {
  for (int round = 0; round < 24; round++) {
    uint64_t c[5], d, b[25];
    for (int x = 0; x < 5; x++) c[x] = a[x] ^ a[x + 5] ^ a[x + 10] ^ a[x + 15] ^ a[x + 20];
    for (int x = 0; x < 5; x++) {
      d = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
      for (int y = 0; y < 25; y += 5) a[y + x] ^= d;
    }
    /* rho + pi: lane (x, y) moves to (y, 2x + 3y), rotated by the triangular offsets */
    unsigned x = 1, y = 0, r = 0;
    b[0] = a[0];
    for (int t = 0; t < 24; t++) {
      r += (unsigned)t + 1;
      unsigned nx = y, ny = (2 * x + 3 * y) % 5;
      b[nx + 5 * ny] = rotl64(a[x + 5 * y], r % 64);
      x = nx;
      y = ny;
    }
    for (int yy = 0; yy < 25; yy += 5)
      for (int xx = 0; xx < 5; xx++) a[yy + xx] = b[yy + xx] ^ (~b[yy + (xx + 1) % 5] & b[yy + (xx + 2) % 5]);
    a[0] ^= KRC[round];
  }
}

/* keccak256 of the nbytes big-endian bytes of v, as a 256-bit big-endian value */
static void vkeccak(val_t* r, const val_t* v, uint32_t nbytes) {
  uint8_t msg[MAXW * 8 + 136];
  for (uint32_t m = 0; m < nbytes; m++) {
    uint32_t bit = 8 * (nbytes - 1 - m);
    msg[m] = (uint8_t)(v->w[bit / 64] >> (bit % 64));
  }
  uint32_t nblk = nbytes / 136 + 1, tot = nblk * 136;
  memset(msg + nbytes, 0, tot - nbytes);
  msg[nbytes] |= 0x01;
  msg[tot - 1] |= 0x80;
  uint64_t st[25];
  memset(st, 0, sizeof(st));
  for (uint32_t blk = 0; blk < nblk; blk++) {
    for (int i = 0; i < 17; i++) {
      uint64_t lane = 0;
      for (int k = 0; k < 8; k++) lane |= (uint64_t)msg[blk * 136 + 8 * i + k] << (8 * k);
      st[i] ^= lane;
    }
    keccak_f1600(st);
  }
  vzero(r);
  for (int m = 0; m < 32; m++) { /* digest byte m is value byte 31 - m */
    uint8_t byte = (uint8_t)(st[m / 8] >> (8 * (m % 8)));
    uint32_t bit = 8 * (31 - m);
    r->w[bit / 64] |= (uint64_t)byte << (bit % 64);
  }
}

static void vadd(val_t* r, const val_t* a, const val_t* b, uint32_t width) {
  unsigned __int128 c = 0;
  for (int i = 0; i < MAXW; i++) {
    c += (unsigned __int128)a->w[i] + b->w[i];
    r->w[i] = (uint64_t)c;
    c >>= 64;
  }
  vmask(r, width);
}

static void vneg(val_t* r, const val_t* a, uint32_t width) {
  val_t t, one;
  for (int i = 0; i < MAXW; i++) t.w[i] = ~a->w[i];
  vzero(&one);
  one.w[0] = 1;
  vadd(r, &t, &one, width);
}

static void vsub(val_t* r, const val_t* a, const val_t* b, uint32_t width) {
  val_t nb;
  vneg(&nb, b, MAXW * 64);
  vadd(r, a, &nb, width);
}

static void vmul(val_t* r, const val_t* a, const val_t* b, uint32_t width, val_t* hi) {
  uint64_t t[2 * MAXW];
  memset(t, 0, sizeof(t));
  int n = nw(width);
  for (int i = 0; i < n; i++) {
    unsigned __int128 c = 0;
    for (int j = 0; j < n; j++) {
      c += (unsigned __int128)a->w[i] * b->w[j] + t[i + j];
      t[i + j] = (uint64_t)c;
      c >>= 64;
    }
    t[i + n] = (uint64_t)c;
  }
  vzero(r);
  for (int i = 0; i < n; i++) r->w[i] = t[i];
  if (hi) {
    /* bits >= width of the full product, shifted down */
    vzero(hi);
    for (uint32_t bit = width; bit < 2 * (uint32_t)n * 64; bit++) {
      if ((t[bit / 64] >> (bit % 64)) & 1) {
        uint32_t k = bit - width;
        if (k < MAXW * 64) hi->w[k / 64] |= 1ull << (k % 64);
      }
    }
  }
  vmask(r, width);
}

static void vshl1(val_t* a) {
  for (int i = MAXW - 1; i > 0; i--) a->w[i] = (a->w[i] << 1) | (a->w[i - 1] >> 63);
  a->w[0] <<= 1;
}

/* long division, bit by bit from the top (any width <= 1024) */
static void vdivrem(const val_t* a, const val_t* b, uint32_t width, val_t* q, val_t* r) {
  vzero(q);
  vzero(r);
  for (int i = (int)width - 1; i >= 0; i--) {
    vshl1(r);
    r->w[0] |= (uint64_t)vbit(a, (uint32_t)i);
    if (!vult(r, b)) {
      val_t t;
      vsub(&t, r, b, MAXW * 64);
      *r = t;
      q->w[i / 64] |= 1ull << (i % 64);
    }
  }
}

static void vshl(val_t* r, const val_t* a, uint64_t s, uint32_t width) {
  vzero(r);
  if (s >= width) return;
  for (uint32_t i = 0; i + s < width; i++)
    if (vbit(a, i)) r->w[(i + s) / 64] |= 1ull << ((i + s) % 64);
}

static void vshr(val_t* r, const val_t* a, uint64_t s, uint32_t width, int fill) {
  vzero(r);
  for (uint32_t i = 0; i < width; i++) {
    uint64_t src = i + s;
    int bit = src < width ? vbit(a, (uint32_t)src) : fill;
    if (bit) r->w[i / 64] |= 1ull << (i % 64);
  }
}

static uint64_t vsmall(const val_t* b, uint32_t cap) {
  for (int i = 1; i < MAXW; i++)
    if (b->w[i]) return cap;
  return b->w[0] < cap ? b->w[0] : cap;
}

/* ---- generator restatement (include/mythgpu.h MG_GEN_*) ---- */
static uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
static uint32_t cand_key(uint64_t idx, uint64_t seed) {
  return mix32((uint32_t)idx ^ mix32((uint32_t)(idx >> 32) ^ (uint32_t)seed ^ mix32((uint32_t)(seed >> 32) + 0x632BE5ABu)));
}
static uint32_t rnd(uint32_t key, uint32_t c, uint32_t j) {
  /* one-multiply finaliser of the (well mixed) candidate key; see MG_GEN_* in mythgpu.h */
  uint32_t x = key ^ (c * 0x9E3779B9u + j * 0x85EBCA6Bu + 0x27D4EB2Fu);
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  return x;
}

static void set_limb32(val_t* v, uint32_t j, uint32_t x) {
  v->w[j / 2] |= (uint64_t)x << (32 * (j % 2));
}

static void from_limbs32(val_t* v, const uint32_t* src, uint32_t L) {
  vzero(v);
  for (uint32_t j = 0; j < L; j++) set_limb32(v, j, src[j]);
}

static void gen_coord(const prog_t* P, uint32_t c, uint32_t key, val_t* out) {
  const uint32_t width = P->coords[4 * c];
  const uint32_t L = (width + 31) / 32;
  uint32_t cc = c;
  uint32_t s[8];
  memcpy(s, P->specs + 8 * c, 32);
  const uint32_t fix_dst = s[0] >> 8; /* 1 + const offset of a (mask, value) fix */
  uint32_t fix_src = 0;
  s[0] &= 0xFFu;
  uint32_t Lg = L;
  int allow_copy = 1, from_mixed = 0, done = 0;
  vzero(out);
  for (int level = 0; level < 2; level++) {
    if (s[0] != 3) break;
    uint32_t h = rnd(key, cc, 0xFFFFu), sel = h & 0xFFFFu;
    /* narrow coordinates (<= 16 bits, MG_GEN_NARROW_BITS): uniform / small value = h >> 16 */
    int narrow = P->coords[4 * cc] <= 16;
    uint32_t pc = (allow_copy && s[4] != NONE) ? s[5] : 0;
    uint32_t pd = s[2] ? s[3] : 0;
    uint32_t ps = s[7] & 0xFFFFu;
    if (sel < pc) {
      cc = s[4];
      memcpy(s, P->specs + 8 * cc, 32);
      fix_src = s[0] >> 8;
      s[0] &= 0xFFu;
      uint32_t Ls = (P->coords[4 * cc] + 31) / 32;
      Lg = Ls < L ? Ls : L;
      allow_copy = 0;
      continue;
    }
    if (sel < pc + pd) {
      s[0] = 2;
      from_mixed = 1;
    } else if (sel < pc + pd + ps) {
      uint32_t bits = (s[7] >> 16) < width ? (s[7] >> 16) : width;
      if (P->coords[4 * cc] < bits) bits = P->coords[4 * cc]; /* a copy keeps the source width */
      for (uint32_t j = 0; j < L; j++) {
        uint32_t v = narrow ? (j == 0 ? h >> 16 : 0u) : rnd(key, cc, j), lo = j * 32;
        v = lo >= bits ? 0u : (bits - lo >= 32 ? v : (v & ((1u << (bits - lo)) - 1u)));
        set_limb32(out, j, v);
      }
      vmask(out, width);
      done = 1;
    } else if (narrow) {
      s[0] = 0xFFu; /* value complete: h >> 16 */
    } else {
      s[0] = 0;
    }
    break;
  }
  const uint32_t Lsrc = (P->coords[4 * cc] + 31) / 32;
  uint32_t limb[64];
  if (done) goto fixes;
  memset(limb, 0, sizeof(limb));
  switch (s[0]) {
    case 0xFFu: /* narrow MIXED draw */
      limb[0] = rnd(key, cc, 0xFFFFu) >> 16;
      break;
    case 2: { /* DICT */
      uint32_t n = s[2];
      uint32_t e = (((rnd(key, cc, 0xFFFFu) >> 16) * n) >> 16);
      const uint32_t* src = P->gconsts + s[1] + e * Lsrc;
      for (uint32_t j = 0; j < Lg; j++) limb[j] = src[j];
      if (from_mixed && s[6]) {
        uint32_t r = rnd(key, cc, 0u);
        if ((r & 0xFFFFu) < s[6]) {
          uint32_t mag = ((r >> 16) & 1u) + 1u;
          int sub = (r >> 17) & 1u;
          uint64_t carry = mag;
          for (uint32_t j = 0; j < Lg; j++) {
            uint64_t t = sub ? ((uint64_t)limb[j] - carry) : ((uint64_t)limb[j] + carry);
            limb[j] = (uint32_t)t;
            carry = sub ? ((t >> 32) & 1u) : (t >> 32);
          }
        }
      }
      break;
    }
    case 1: { /* RANGE */
      uint32_t span = s[2], r = rnd(key, cc, 0);
      uint32_t off = span ? (uint32_t)(((uint64_t)r * span) >> 32) : r;
      uint64_t carry = off;
      for (uint32_t j = 0; j < Lg; j++) {
        uint64_t t = (uint64_t)P->gconsts[s[1] + j] + carry;
        limb[j] = (uint32_t)t;
        carry = t >> 32;
      }
      break;
    }
    case 4: { /* ALIGNED */
      uint32_t cnt = s[3], r = rnd(key, cc, 0);
      uint64_t m = cnt ? (((uint64_t)r * cnt) >> 32) : r;
      uint32_t sh = s[2];
      uint64_t carry = 0;
      for (uint32_t j = 0; j < Lg; j++) {
        int32_t bit0 = (int32_t)(j * 32) - (int32_t)sh;
        uint32_t mw;
        if (bit0 <= -32 || bit0 >= 64) mw = 0;
        else if (bit0 < 0) mw = (uint32_t)(m << (-bit0));
        else mw = (uint32_t)(m >> bit0);
        uint64_t t = (uint64_t)P->gconsts[s[1] + j] + mw + carry;
        limb[j] = (uint32_t)t;
        carry = t >> 32;
      }
      break;
    }
    case 5: /* FIXED */
      for (uint32_t j = 0; j < Lg; j++) limb[j] = P->gconsts[s[1] + j];
      break;
    default: /* UNIFORM / LAZY */
      for (uint32_t j = 0; j < Lg; j++) limb[j] = rnd(key, cc, j);
      break;
  }
  /* a copy is the source's value: masked to the source width, then truncated / zero-extended */
  if (cc != c && Lg == Lsrc && (P->coords[4 * cc] & 31u)) limb[Lg - 1] &= (1u << (P->coords[4 * cc] & 31u)) - 1u;
  from_limbs32(out, limb, Lg);
  vmask(out, width);
fixes:
  /* fixed bits (v & ~mask) | value: the copied source's fix, then this coordinate's */
  if (cc != c && fix_src) {
    const uint32_t* f = P->gconsts + (fix_src - 1);
    for (uint32_t j = 0; j < Lg; j++) {
      uint32_t x = (uint32_t)(out->w[j / 2] >> (32 * (j % 2)));
      x = (x & ~f[j]) | f[Lsrc + j];
      out->w[j / 2] = (out->w[j / 2] & ~(0xFFFFFFFFull << (32 * (j % 2)))) | ((uint64_t)x << (32 * (j % 2)));
    }
  }
  if (fix_dst) {
    const uint32_t* f = P->gconsts + (fix_dst - 1);
    for (uint32_t j = 0; j < L; j++) {
      uint32_t x = (uint32_t)(out->w[j / 2] >> (32 * (j % 2)));
      x = (x & ~f[j]) | f[L + j];
      out->w[j / 2] = (out->w[j / 2] & ~(0xFFFFFFFFull << (32 * (j % 2)))) | ((uint64_t)x << (32 * (j % 2)));
    }
  }
}

/* ---- evaluation ---- */
typedef struct {
  uint32_t table;
  val_t key, val;
} entry_t;

typedef struct {
  const prog_t* P;
  val_t* vals;       /* per node */
  entry_t* entries;  /* per-candidate tables, in SSA order */
  int n_entries;
  uint32_t key;
  const uint32_t* soa; /* optional explicit coordinates (rows x n) */
  uint64_t soa_n, soa_i;
  const uint32_t* coord_row;
} ctx_t;

static void coord_value(ctx_t* X, uint32_t c, val_t* out) {
  const uint32_t width = X->P->coords[4 * c];
  if (X->soa) {
    uint32_t L = (width + 31) / 32;
    vzero(out);
    for (uint32_t j = 0; j < L; j++) set_limb32(out, j, X->soa[(uint64_t)(X->coord_row[c] + j) * X->soa_n + X->soa_i]);
    vmask(out, width);
  } else {
    gen_coord(X->P, c, X->key, out);
  }
}

static void site_lookup(ctx_t* X, uint32_t table, const val_t* key, const val_t* dflt, val_t* out) {
  for (int e = 0; e < X->n_entries; e++) {
    if (X->entries[e].table == table && veq(&X->entries[e].key, key)) {
      *out = X->entries[e].val;
      return;
    }
  }
  *out = *dflt;
  entry_t* n = &X->entries[X->n_entries++];
  n->table = table;
  n->key = *key;
  n->val = *dflt;
}

static int eval_candidate(ctx_t* X) {
  const prog_t* P = X->P;
  X->n_entries = 0;
  for (uint32_t i = 0; i < P->n_nodes; i++) {
    const node_t* n = &P->nodes[i];
    val_t* r = &X->vals[i];
    const val_t *A = n->a != NONE && n->a < i ? &X->vals[n->a] : NULL;
    const val_t *B = n->b != NONE && n->b < i ? &X->vals[n->b] : NULL;
    const val_t *Cc = n->c != NONE && n->c < i ? &X->vals[n->c] : NULL;
    const uint32_t W = n->width;
    uint32_t wa = (n->a != NONE && n->a < i) ? P->nodes[n->a].width : 0;
    vzero(r);
    switch (n->op) {
      case OP_CONST: from_limbs32(r, P->consts + n->p0, (W + 31) / 32); vmask(r, W); break;
      case OP_VAR: coord_value(X, n->p0, r); break;
      case OP_ADD: vadd(r, A, B, W); break;
      case OP_SUB: vsub(r, A, B, W); break;
      case OP_MUL: vmul(r, A, B, W, NULL); break;
      case OP_UDIV: case OP_UREM: {
        val_t q, rm;
        if (viszero(B)) {
          if (n->op == OP_UDIV) { for (int k = 0; k < MAXW; k++) r->w[k] = ~0ull; vmask(r, W); }
          else *r = *A;
        } else {
          vdivrem(A, B, W, &q, &rm);
          *r = n->op == OP_UDIV ? q : rm;
        }
        break;
      }
      case OP_SDIV: case OP_SREM: case OP_SMOD: {
        int sa = vbit(A, W - 1), sb = vbit(B, W - 1);
        val_t aa = *A, bb = *B, q, rm;
        if (sa) vneg(&aa, A, W);
        if (sb) vneg(&bb, B, W);
        if (viszero(&bb)) {
          vzero(&q);
          for (int k = 0; k < MAXW; k++) q.w[k] = ~0ull;
          vmask(&q, W);
          rm = aa;
        } else {
          vdivrem(&aa, &bb, W, &q, &rm);
        }
        if (n->op == OP_SDIV) {
          if (sa ^ sb) vneg(r, &q, W); else *r = q;
        } else if (n->op == OP_SREM) {
          if (sa) vneg(r, &rm, W); else *r = rm;
        } else {
          if (viszero(&rm) || (!sa && !sb)) *r = rm;
          else if (sa && !sb) { val_t t; vneg(&t, &rm, W); vadd(r, &t, B, W); }
          else if (!sa && sb) vadd(r, &rm, B, W);
          else vneg(r, &rm, W);
        }
        break;
      }
      case OP_AND: for (int k = 0; k < MAXW; k++) r->w[k] = A->w[k] & B->w[k]; break;
      case OP_OR: for (int k = 0; k < MAXW; k++) r->w[k] = A->w[k] | B->w[k]; break;
      case OP_XOR: for (int k = 0; k < MAXW; k++) r->w[k] = A->w[k] ^ B->w[k]; break;
      case OP_NOT: for (int k = 0; k < MAXW; k++) r->w[k] = ~A->w[k]; vmask(r, W); break;
      case OP_NEG: vneg(r, A, W); break;
      case OP_SHL: vshl(r, A, vsmall(B, W), W); break;
      case OP_LSHR: vshr(r, A, vsmall(B, W), W, 0); break;
      case OP_ASHR: vshr(r, A, vsmall(B, W), W, vbit(A, W - 1)); break;
      case OP_CONCAT: {
        uint32_t wb = P->nodes[n->b].width;
        vshl(r, A, wb, W);
        for (int k = 0; k < MAXW; k++) r->w[k] |= B->w[k];
        break;
      }
      case OP_EXTRACT: vshr(r, A, n->p0, wa, 0); vmask(r, W); break;
      case OP_ZEXT: *r = *A; break;
      case OP_SEXT: {
        *r = *A;
        if (vbit(A, wa - 1))
          for (uint32_t k = wa; k < W; k++) r->w[k / 64] |= 1ull << (k % 64);
        break;
      }
      case OP_ITE: *r = A->w[0] ? *B : *Cc; break;
      case OP_EQ: r->w[0] = veq(A, B); break;
      case OP_ULT: r->w[0] = vult(A, B); break;
      case OP_ULE: r->w[0] = !vult(B, A); break;
      case OP_SLT: case OP_SLE: {
        int sa = vbit(A, wa - 1), sb = vbit(B, wa - 1);
        int lt = sa != sb ? sa : vult(A, B);
        r->w[0] = n->op == OP_SLT ? lt : (lt || veq(A, B));
        break;
      }
      case OP_UMUL_NOOVF: {
        val_t lo, hi;
        vmul(&lo, A, B, wa, &hi);
        r->w[0] = viszero(&hi);
        break;
      }
      case OP_ARR_VAR: case OP_ARR_K: case OP_ARR_STORE: break;
      case OP_SELECT: {
        /* base read first (it registers its table entry), then the store chain */
        uint32_t arr = n->a;
        uint32_t chain[4096];
        int depth = 0;
        while (P->nodes[arr].op == OP_ARR_STORE && depth < 4096) {
          chain[depth++] = arr;
          arr = P->nodes[arr].a;
        }
        val_t base;
        if (P->nodes[arr].op == OP_ARR_K) {
          base = X->vals[P->nodes[arr].a];
        } else {
          val_t dflt;
          coord_value(X, n->p0, &dflt);
          site_lookup(X, P->nodes[arr].p0, B, &dflt, &base);
        }
        *r = base;
        for (int d = depth - 1; d >= 0; d--) { /* oldest store first; newest decides last */
          const node_t* st = &P->nodes[chain[d]];
          if (veq(B, &X->vals[st->b])) *r = X->vals[st->c];
        }
        break;
      }
      case OP_UFAPP: {
        val_t dflt;
        if (n->p2 != NONE) dflt = X->vals[n->p2];
        else coord_value(X, n->p1, &dflt);
        site_lookup(X, n->p0, A, &dflt, r);
        break;
      }
      case OP_EXP: {
        val_t acc, sq;
        vzero(&acc);
        acc.w[0] = 1;
        for (int bit = (int)W - 1; bit >= 0; bit--) {
          vmul(&sq, &acc, &acc, W, NULL);
          acc = sq;
          if (vbit(B, (uint32_t)bit)) {
            vmul(&sq, &acc, A, W, NULL);
            acc = sq;
          }
        }
        *r = acc;
        break;
      }
      case OP_KECCAK:
        if (A) vkeccak(r, A, n->p0);
        else { val_t z; vzero(&z); vkeccak(r, &z, 0); }
        break;
      default:
        return -1;
    }
  }
  for (uint32_t k = 0; k < P->n_roots; k++)
    if (!X->vals[P->roots[k]].w[0]) return 0;
  return 1;
}

static int parse(prog_t* P, const uint32_t* w, size_t n, const uint32_t* gen, size_t gen_n) {
  if (n < 16 || w[0] != 0x3150474Du) return -1;
  P->n_nodes = w[2];
  P->n_roots = w[3];
  P->n_coords = w[4];
  P->n_tables = w[5];
  P->n_consts = w[6];
  uint32_t n_watch = w[7];
  size_t pos = 16;
  P->nodes = (const node_t*)(w + pos);
  pos += 8ull * P->n_nodes;
  P->roots = w + pos;
  pos += P->n_roots;
  P->coords = w + pos;
  pos += 4ull * P->n_coords;
  P->tables = w + pos;
  pos += 4ull * P->n_tables;
  pos += n_watch;
  P->consts = w + pos;
  pos += P->n_consts;
  if (pos != n) return -1;
  for (uint32_t i = 0; i < P->n_nodes; i++)
    if (P->nodes[i].width > MAXW * 64) return -2;
  if (gen) {
    if (gen_n < 4 || gen[0] != 0x314E4547u || gen[1] != P->n_coords) return -1;
    P->gen_n = gen[1];
    P->specs = gen + 4;
    P->gconsts = gen + 4 + 8ull * gen[1];
  }
  return 0;
}

/* Evaluate candidates [start, start+count) from the generator; returns 0 or <0.
 * verdicts (nullable): count bytes. */
int bv_search(const uint32_t* prog, size_t prog_words, const uint32_t* gen, size_t gen_words, uint64_t seed,
              uint64_t start, uint64_t count, int threads, uint64_t* first_hit, uint64_t* n_hits,
              uint8_t* verdicts) {
  prog_t P;
  int rc = parse(&P, prog, prog_words, gen, gen_words);
  if (rc) return rc;
  uint64_t best = ~0ull, hits = 0;
  int err = 0;
#ifdef _OPENMP
  if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel reduction(min : best) reduction(+ : hits) reduction(| : err)
#endif
  {
    ctx_t X;
    memset(&X, 0, sizeof(X));
    X.P = &P;
    X.vals = (val_t*)malloc(sizeof(val_t) * (P.n_nodes + 1));
    X.entries = (entry_t*)malloc(sizeof(entry_t) * (P.n_nodes + 1));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 256)
#endif
    for (int64_t i = 0; i < (int64_t)count; i++) {
      uint64_t idx = start + (uint64_t)i;
      X.key = cand_key(idx, seed);
      int v = eval_candidate(&X);
      if (v < 0) {
        err |= 1;
        continue;
      }
      if (verdicts) verdicts[i] = (uint8_t)v;
      if (v) {
        hits++;
        if (idx < best) best = idx;
      }
    }
    free(X.vals);
    free(X.entries);
  }
  if (err) return -3;
  *first_hit = best;
  *n_hits = hits;
  return 0;
}

/* Evaluate explicit assignments (SoA [row][n], as mg_eval); optional per-node dump
 * of node `watch_node` values (dump: n x MAXW 64-bit words). */
int bv_eval(const uint32_t* prog, size_t prog_words, const uint32_t* soa, uint64_t n, uint8_t* verdicts) {
  prog_t P;
  int rc = parse(&P, prog, prog_words, NULL, 0);
  if (rc) return rc;
  uint32_t* rows = (uint32_t*)malloc(sizeof(uint32_t) * (P.n_coords + 1));
  uint32_t acc = 0;
  for (uint32_t c = 0; c < P.n_coords; c++) {
    rows[c] = acc;
    acc += (P.coords[4 * c] + 31) / 32;
  }
  ctx_t X;
  memset(&X, 0, sizeof(X));
  X.P = &P;
  X.vals = (val_t*)malloc(sizeof(val_t) * (P.n_nodes + 1));
  X.entries = (entry_t*)malloc(sizeof(entry_t) * (P.n_nodes + 1));
  X.soa = soa;
  X.soa_n = n;
  X.coord_row = rows;
  int bad = 0;
  for (uint64_t i = 0; i < n; i++) {
    X.soa_i = i;
    int v = eval_candidate(&X);
    if (v < 0) bad = 1;
    verdicts[i] = (uint8_t)(v > 0);
  }
  free(X.vals);
  free(X.entries);
  free(rows);
  return bad ? -3 : 0;
}
