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
  uint32_t n_watch;
  const uint32_t* watch; /* node ids whose values a model read-back returns */
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
  uint64_t br = 0;
  for (int i = 0; i < MAXW; i++) {
    const uint64_t x = a->w[i], y = b->w[i];
    r->w[i] = x - y - br;
    br = (x < y) || (x - y < br);
  }
  vmask(r, width);
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
  int small = b->w[0] != 0;
  for (int i = 1; i < MAXW && small; i++) small = b->w[i] == 0;
  if (small) { /* a one-word divisor: schoolbook division by 64-bit digits */
    unsigned __int128 rem = 0;
    for (int i = nw(width) - 1; i >= 0; i--) {
      const unsigned __int128 cur = (rem << 64) | a->w[i];
      q->w[i] = (uint64_t)(cur / b->w[0]);
      rem = cur % b->w[0];
    }
    r->w[0] = (uint64_t)rem;
    return;
  }
  int top = (int)width - 1; /* the dividend's leading zeros leave r = 0 and their quotient bits 0 */
  while (top >= 0 && !vbit(a, (uint32_t)top)) top--;
  for (int i = top; i >= 0; i--) {
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

/* shifts by whole words and a bit remainder; the operand is masked to the width first */
static void vshl(val_t* r, const val_t* a, uint64_t s, uint32_t width) {
  vzero(r);
  if (s >= width) return;
  val_t t = *a;
  vmask(&t, width);
  const int q = (int)(s / 64), b = (int)(s % 64);
  for (int i = MAXW - 1; i >= q; i--) {
    uint64_t x = t.w[i - q] << b;
    if (b && i - q >= 1) x |= t.w[i - q - 1] >> (64 - b);
    r->w[i] = x;
  }
  vmask(r, width);
}

static void vshr(val_t* r, const val_t* a, uint64_t s, uint32_t width, int fill) {
  vzero(r);
  val_t t = *a;
  vmask(&t, width);
  if (s < width) {
    const int q = (int)(s / 64), b = (int)(s % 64);
    for (int i = 0; i + q < MAXW; i++) {
      uint64_t x = t.w[i + q] >> b;
      if (b && i + q + 1 < MAXW) x |= t.w[i + q + 1] << (64 - b);
      r->w[i] = x;
    }
  }
  if (fill) /* bits [width - s, width) take the sign */
    for (uint32_t i = s < width ? width - (uint32_t)s : 0; i < width; i++) r->w[i / 64] |= 1ull << (i % 64);
  vmask(r, width);
}

static uint64_t vsmall(const val_t* b, uint32_t cap) {
  for (int i = 1; i < MAXW; i++)
    if (b->w[i]) return cap;
  return b->w[0] < cap ? b->w[0] : cap;
}

/* ---- generator restatement (include/mythgpu.h, format GEN3) ---- */
static uint64_t fmix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xFF51AFD7ED558CCDull;
  x ^= x >> 33;
  x *= 0xC4CEB9FE1A85EC53ull;
  x ^= x >> 33;
  return x;
}

typedef struct {
  uint32_t klo, khi, glo, ghi;
} keys_t;

static void make_keys(uint64_t idx, uint64_t seed, keys_t* k) {
  const uint64_t G = fmix64((idx >> 6) ^ fmix64(seed ^ 0xBB67AE8584CAA73Bull));
  const uint64_t K = G ^ fmix64((idx & 63u) ^ fmix64(seed ^ 0x6A09E667F3BCC908ull));
  k->klo = (uint32_t)K;
  k->khi = (uint32_t)(K >> 32);
  k->glo = (uint32_t)G;
  k->ghi = (uint32_t)(G >> 32);
}

static uint32_t salt(uint32_t c, uint32_t j) { return c * 0x9E3779B9u + j * 0x85EBCA6Bu + 0x27D4EB2Fu; }

static uint32_t fin(uint32_t x) {
  x ^= x >> 16;
  x = (x & 0xFFFFFFu) * 0x9E3779u; /* 24 x 24 -> low 32 bits */
  x ^= x >> 15;
  return x;
}

static uint32_t rnd(const keys_t* k, uint32_t c, uint32_t j) { return fin(k->klo ^ salt(c, j)) + k->khi; }
static uint32_t wsel(const keys_t* k, uint32_t c) { return (k->glo ^ salt(c, 0xFFFEu)) * 0x9E3779B1u + k->ghi; }

/* the raw limbs of a UNIFORM draw: u0 = rnd(c, 0), u1 = rnd(c, 1), then
   u_j = low 32 bits of ((u_{j-1} : u_{j-2}) >> s_j) + u_{j-2}  (mod 2^32),
   s_j = (7j + 3) mod 31 + 1 */
static void uniform_raw(const keys_t* k, uint32_t c, uint32_t L, uint32_t* u) {
  for (uint32_t j = 0; j < L; j++) {
    if (j < 2) {
      u[j] = rnd(k, c, j);
    } else {
      const uint64_t pair = ((uint64_t)u[j - 1] << 32) | u[j - 2];
      u[j] = (uint32_t)(pair >> ((7u * j + 3u) % 31u + 1u)) + u[j - 2];
    }
  }
}

static void set_limb32(val_t* v, uint32_t j, uint32_t x) {
  v->w[j / 2] |= (uint64_t)x << (32 * (j % 2));
}

static uint32_t get_limb32(const val_t* v, uint32_t j) { return (uint32_t)(v->w[j / 2] >> (32 * (j % 2))); }

static void from_limbs32(val_t* v, const uint32_t* src, uint32_t L) {
  vzero(v);
  for (uint32_t j = 0; j < L; j++) set_limb32(v, j, src[j]);
}

static void mask_limbs(uint32_t* limb, uint32_t L, uint32_t width) {
  if (width & 31u) limb[L - 1] &= (1u << (width & 31u)) - 1u;
}

/* lo + off over L limbs (carry out dropped) */
static void add_small(uint32_t* out, const uint32_t* lo, uint64_t off, uint32_t L) {
  uint64_t carry = off;
  for (uint32_t j = 0; j < L; j++) {
    uint64_t t = (uint64_t)lo[j] + (carry & 0xFFFFFFFFull);
    carry = (carry >> 32) + (t >> 32);
    out[j] = (uint32_t)t;
  }
}

struct ctx;
static void coord_value(struct ctx* X, uint32_t c, val_t* out);

/* generated value of coordinate c (GEN3 semantics in include/mythgpu.h) into L limbs */
static void gen_value(struct ctx* X, const prog_t* P, const keys_t* k, uint32_t c, uint32_t* limb) {
  const uint32_t width = P->coords[4 * c];
  const uint32_t L = (width + 31) / 32;
  const uint32_t* s = P->specs + 8 * c;
  const uint32_t kind = s[0] & 0xFFu, fix = s[0] >> 8;
  memset(limb, 0, 4 * L);
  switch (kind) {
    case 1: { /* RANGE */
      const uint32_t span = s[2], r = rnd(k, c, 0);
      add_small(limb, P->gconsts + s[1], span ? (((uint64_t)r * span) >> 32) : r, L);
      break;
    }
    case 2: { /* DICT */
      const uint32_t e = ((rnd(k, c, 0xFFFFu) >> 16) * s[2]) >> 16;
      memcpy(limb, P->gconsts + s[1] + e * L, 4 * L);
      break;
    }
    case 4: { /* ALIGNED */
      const uint32_t cnt = s[3], r = rnd(k, c, 0);
      const uint64_t m = cnt ? (((uint64_t)r * cnt) >> 32) : r;
      const uint32_t sh = s[2];
      uint64_t carry = 0;
      for (uint32_t j = 0; j < L; j++) {
        const int32_t bit0 = (int32_t)(j * 32) - (int32_t)sh;
        uint32_t mw;
        if (bit0 <= -32 || bit0 >= 64) mw = 0;
        else if (bit0 < 0) mw = (uint32_t)(m << (-bit0));
        else mw = (uint32_t)(m >> bit0);
        const uint64_t t = (uint64_t)P->gconsts[s[1] + j] + mw + carry;
        limb[j] = (uint32_t)t;
        carry = t >> 32;
      }
      break;
    }
    case 5: /* FIXED */
      memcpy(limb, P->gconsts + s[1], 4 * L);
      break;
    case 3: { /* MIXED: one alternative per aligned group of 64 indices */
      const uint32_t ws = wsel(k, c), sel = ws >> 16;
      const uint32_t pc = s[4] != NONE ? (s[3] & 0xFFFFu) : 0u;
      const uint32_t pd = s[2] ? (s[3] >> 16) : 0u;
      const uint32_t ps = s[5] & 0xFFFFu;
      const uint32_t h = rnd(k, c, 0xFFFFu);
      const int narrow = width <= 16;
      int with_delta = 0;
      if (sel < pc) { /* COPY: the source's final value */
        val_t src;
        coord_value(X, s[4], &src);
        for (uint32_t j = 0; j < L; j++) limb[j] = get_limb32(&src, j);
        with_delta = 1;
      } else if (sel < pc + pd) { /* DICT */
        const uint32_t e = ((h >> 16) * s[2]) >> 16;
        memcpy(limb, P->gconsts + s[1] + e * L, 4 * L);
        with_delta = 1;
      } else {
        const uint32_t small = sel < pc + pd + ps;
        uint32_t bits = small ? (s[5] >> 16) : width;
        if (bits > width) bits = width;
        if (narrow) {
          limb[0] = h & 0xFFFFu;
        } else {
          uniform_raw(k, c, L, limb);
        }
        for (uint32_t j = 0; j < L; j++) {
          const uint32_t lo = 32 * j;
          limb[j] = lo >= bits ? 0u : (bits - lo >= 32 ? limb[j] : (limb[j] & ((1u << (bits - lo)) - 1u)));
        }
      }
      if (with_delta && (ws & 0xFFFFu) < s[6]) {
        const uint32_t mag = 1u + (h & 1u);
        const int sub = (h >> 1) & 1u;
        uint64_t cy = mag;
        for (uint32_t j = 0; j < L; j++) {
          const uint64_t t = sub ? ((uint64_t)limb[j] - cy) : ((uint64_t)limb[j] + cy);
          limb[j] = (uint32_t)t;
          cy = sub ? ((t >> 32) & 1u) : (t >> 32);
        }
      }
      mask_limbs(limb, L, width);
      if (s[7]) { /* clamp into [lo, lo + span) */
        const uint32_t* lo = P->gconsts + (s[7] - 1);
        const uint32_t span = lo[L];
        uint64_t br = 0;
        uint32_t hi_or = 0, t0 = 0;
        for (uint32_t j = 0; j < L; j++) {
          const uint64_t t = (uint64_t)limb[j] - lo[j] - br;
          br = (t >> 32) & 1u;
          if (j == 0) t0 = (uint32_t)t;
          else hi_or |= (uint32_t)t;
        }
        const int in = !br && !hi_or && (span == 0 || t0 < span);
        if (!in) add_small(limb, lo, span ? (((uint64_t)limb[0] * span) >> 32) : limb[0], L);
      }
      break;
    }
    default: /* UNIFORM / LAZY */
      uniform_raw(k, c, L, limb);
      break;
  }
  mask_limbs(limb, L, width);
  if (fix) { /* fixed bits: (v & ~mask) | value */
    const uint32_t* f = P->gconsts + (fix - 1);
    for (uint32_t j = 0; j < L; j++) limb[j] = (limb[j] & ~f[j]) | f[L + j];
  }
}

/* ---- evaluation ---- */
typedef struct {
  uint32_t table;
  val_t key, val;
} entry_t;

typedef struct ctx {
  const prog_t* P;
  val_t* vals;       /* per node */
  entry_t* entries;  /* per-candidate tables, in SSA order */
  int n_entries;
  keys_t keys;
  val_t* cvals;      /* per coordinate: generated value (search mode), memoised per candidate */
  uint8_t* cdone;
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
    return;
  }
  if (!X->cdone[c]) {
    uint32_t limb[MAXW * 2];
    gen_value(X, X->P, &X->keys, c, limb);
    from_limbs32(&X->cvals[c], limb, (width + 31) / 32);
    X->cdone[c] = 1;
  }
  *out = X->cvals[c];
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
  if (X->cdone) memset(X->cdone, 0, P->n_coords);
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
          if (n->p1 != NONE) dflt = X->vals[n->p1]; /* lazy default (an AUX word's byte) */
          else coord_value(X, n->p0, &dflt);
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
  if (n < 16 || w[0] != 0x3150474Du || w[1] != 2u) return -1;
  P->n_nodes = w[2];
  P->n_roots = w[3];
  P->n_coords = w[4];
  P->n_tables = w[5];
  P->n_consts = w[6];
  uint32_t n_watch = w[7];
  P->n_watch = n_watch;
  size_t pos = 16;
  P->nodes = (const node_t*)(w + pos);
  pos += 8ull * P->n_nodes;
  P->roots = w + pos;
  pos += P->n_roots;
  P->coords = w + pos;
  pos += 4ull * P->n_coords;
  P->tables = w + pos;
  pos += 4ull * P->n_tables;
  P->watch = w + pos;
  pos += n_watch;
  P->consts = w + pos;
  pos += P->n_consts;
  if (pos != n) return -1;
  for (uint32_t i = 0; i < P->n_nodes; i++)
    if (P->nodes[i].width > MAXW * 64) return -2;
  if (gen) {
    if (gen_n < 4 || gen[0] != 0x334E4547u || gen[1] != P->n_coords) return -1;
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
    X.cvals = (val_t*)malloc(sizeof(val_t) * (P.n_coords + 1));
    X.cdone = (uint8_t*)malloc(P.n_coords + 1);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 256)
#endif
    for (int64_t i = 0; i < (int64_t)count; i++) {
      uint64_t idx = start + (uint64_t)i;
      make_keys(idx, seed, &X.keys);
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
    free(X.cvals);
    free(X.cdone);
  }
  if (err) return -3;
  *first_hit = best;
  *n_hits = hits;
  return 0;
}

/* Evaluate explicit assignments (SoA [row][n], as mg_eval); optional per-node dump
 * of node `watch_node` values (dump: n x MAXW 64-bit words). */
int bv_eval_watch(const uint32_t* prog, size_t prog_words, const uint32_t* soa, uint64_t n, uint8_t* verdicts,
                  uint32_t* watch_out);

int bv_eval(const uint32_t* prog, size_t prog_words, const uint32_t* soa, uint64_t n, uint8_t* verdicts) {
  return bv_eval_watch(prog, prog_words, soa, n, verdicts, NULL);
}

/* ... and (watch_out non-null) the model read-back mg_eval returns: watch node k's value as
 * ceil(width/32) little-endian limb rows of n uint32, the watch list in order
 * (laser/smt/model.py:45-59, Model.eval of each watched term). */
int bv_eval_watch(const uint32_t* prog, size_t prog_words, const uint32_t* soa, uint64_t n, uint8_t* verdicts,
                  uint32_t* watch_out) {
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
    if (watch_out) {
      uint64_t row = 0;
      for (uint32_t k = 0; k < P.n_watch; k++) {
        const uint32_t id = P.watch[k];
        if (id >= P.n_nodes) { bad = 1; break; }
        const uint32_t L = (P.nodes[id].width + 31) / 32;
        for (uint32_t j = 0; j < L; j++) watch_out[(row + j) * n + i] = get_limb32(&X.vals[id], j);
        row += L;
      }
    }
  }
  free(X.vals);
  free(X.entries);
  free(rows);
  return bad ? -3 : 0;
}

/* The generated coordinates of candidates [start, start+n) as an SoA buffer ([row][n], the
 * mg_eval layout; LAZY coordinates, whose values the program supplies, stay zero): lets a
 * test run another evaluator (oracle/kops.py over the engine's specialised program) on
 * exactly the candidates the generator draws. */
int bv_gen_soa(const uint32_t* prog, size_t prog_words, const uint32_t* gen, size_t gen_words, uint64_t seed,
               uint64_t start, uint64_t n, uint32_t* soa) {
  prog_t P;
  int rc = parse(&P, prog, prog_words, gen, gen_words);
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
  X.cvals = (val_t*)malloc(sizeof(val_t) * (P.n_coords + 1));
  X.cdone = (uint8_t*)malloc(P.n_coords + 1);
  memset(soa, 0, sizeof(uint32_t) * (size_t)acc * n);
  for (uint64_t i = 0; i < n; i++) {
    make_keys(start + i, seed, &X.keys);
    memset(X.cdone, 0, P.n_coords);
    for (uint32_t c = 0; c < P.n_coords; c++) {
      if ((P.specs[8 * c] & 0xFFu) == 6u) continue; /* LAZY */
      val_t v;
      coord_value(&X, c, &v);
      const uint32_t L = (P.coords[4 * c] + 31) / 32;
      for (uint32_t j = 0; j < L; j++) soa[(uint64_t)(rows[c] + j) * n + i] = get_limb32(&v, j);
    }
  }
  free(X.cvals);
  free(X.cdone);
  free(rows);
  return 0;
}
