/*
 * mythgpu.h — C-ABI of the MI355X batched bit-vector evaluation engine.
 *
 * This is the drop-in boundary for ONE hot path of the reference
 * (strawberrylady99/mythril v0.22.7): the satisfiability queries LASER sends to
 * z3 through `get_model` (mythril/support/model.py:15-49) and the model
 * evaluation z3 performs for `Model.eval` (mythril/laser/smt/model.py:45-59).
 * The reference reaches z3 through z3py/ctypes (libz3); this library is loaded
 * the same way (ctypes) by `mythril_amd/native.py`.
 *
 * Entry points and the reference interface each one replaces:
 *
 *   mg_init / mg_shutdown     z3 context creation (implicit in z3py import,
 *                             mythril/laser/smt/solver/__init__.py:1-9)
 *   mg_program_load           Solver.add / Optimize.add of the constraint list
 *                             (mythril/laser/smt/solver/solver.py:28-45,
 *                             mythril/support/model.py:38-39): the flattened
 *                             SSA program of the whole conjunction
 *   mg_search                 Optimize.check() for SAT instances
 *                             (mythril/support/model.py:44,
 *                             solver.py:47-57): first satisfying candidate index
 *   mg_eval / mg_eval_generated
 *                             ModelRef.eval(expr, model_completion=True)
 *                             (mythril/laser/smt/model.py:45-59) batched over
 *                             N assignments; also Solver.model() materialisation
 *                             (solver.py:59-64) of a search hit
 *   mg_keccak256              ethereum.utils.sha3 used for concrete SHA3
 *                             (mythril/laser/ethereum/keccak_function_manager.py:44-57,
 *                             mythril/analysis/solver.py:146)
 *   mg_stats                  SolverStatistics (laser/smt/solver/solver_statistics.py:8-43)
 *   mg_last_error             z3 exceptions -> here: an error string; the host
 *                             maps any error to "unknown" (never to unsat)
 *
 * Conventions: every function returns 0 on success and a negative MG_E_* code on
 * failure (no C++ exception crosses the ABI). Host buffers are caller-owned.
 * Functions with the `_dev` suffix take device pointers already resident in HBM
 * (used by the benchmark so that the timed region excludes PCIe).
 * Multi-GPU: mg_init's mask opens several GPUs in one process, and mg_search /
 * mg_jit_search split a large call over them inside the shim (host min/sum of 16 bytes
 * per device, no collective).  One process per GPU also works (mask = one bit): the
 * caller then shards the index space and reduces the first hit itself (bench.py under
 * torch.distributed.run: one all-reduce(MIN) over RCCL per epoch).
 */
#ifndef MYTHGPU_H
#define MYTHGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes ---------------------------------------------------- */
#define MG_OK 0
#define MG_E_INVALID (-1)      /* malformed program / argument */
#define MG_E_UNSUPPORTED (-2)  /* operator or width outside the engine: fall back to z3 */
#define MG_E_HIP (-3)          /* HIP runtime error */
#define MG_E_NODEVICE (-4)     /* no usable gfx950 device */
#define MG_E_NOMEM (-5)
#define MG_E_NOTINIT (-6)

/* ---- program format v1 ---------------------------------------------- *
 * Little-endian uint32 words:
 *   header[16]  : MG_MAGIC, MG_VERSION, n_nodes, n_roots, n_coords, n_tables,
 *                 n_const_words, n_watch, 0...
 *   nodes       : n_nodes x 8 words {op, width, a, b, c, p0, p1, p2}
 *                 operands a/b/c are indices of EARLIER nodes (SSA order)
 *   roots       : n_roots node indices (Bool nodes; the query is their AND)
 *   coords      : n_coords x 4 words {width, kind, node, table}
 *   tables      : n_tables x 4 words {kind, key_width, val_width, 0}
 *   watch       : n_watch node indices whose values mg_eval dumps
 *   consts      : n_const_words (little-endian 32-bit limbs)
 * A value of width w occupies ceil(w/32) limbs, limb 0 least significant,
 * unused high bits zero.  Bool = width 1.
 */
#define MG_MAGIC 0x3150474Du /* "MGP1" */
#define MG_VERSION 2u  /* v2: SELECT p1 = lazy default node, AUX coordinates */
#define MG_NONE 0xFFFFFFFFu
#define MG_MAX_WIDTH 32768u

enum mg_op {
  MG_OP_CONST = 0,      /* p0 = const word offset */
  MG_OP_VAR = 1,        /* p0 = coord index */
  MG_OP_ADD = 2,
  MG_OP_SUB = 3,
  MG_OP_MUL = 4,
  MG_OP_UDIV = 5,
  MG_OP_UREM = 6,
  MG_OP_SDIV = 7,
  MG_OP_SREM = 8,
  MG_OP_SMOD = 9,
  MG_OP_AND = 10,
  MG_OP_OR = 11,
  MG_OP_XOR = 12,
  MG_OP_NOT = 13,
  MG_OP_NEG = 14,
  MG_OP_SHL = 15,
  MG_OP_LSHR = 16,
  MG_OP_ASHR = 17,
  MG_OP_CONCAT = 18,    /* a = high part, b = low part */
  MG_OP_EXTRACT = 19,   /* p0 = lo; width = hi-lo+1 */
  MG_OP_ZEXT = 20,
  MG_OP_SEXT = 21,
  MG_OP_ITE = 22,       /* a = Bool condition */
  MG_OP_EQ = 23,
  MG_OP_ULT = 24,
  MG_OP_ULE = 25,
  MG_OP_SLT = 26,
  MG_OP_SLE = 27,
  MG_OP_UMUL_NOOVF = 28,
  MG_OP_ARR_VAR = 29,   /* array-sorted: p0 = table */
  MG_OP_ARR_K = 30,     /* array-sorted: a = default value */
  MG_OP_ARR_STORE = 31, /* array-sorted: a = array, b = index, c = value */
  MG_OP_SELECT = 32,    /* a = array, b = index, p0 = coord of the base read (or MG_NONE),
                           p1 = node giving the base read's default (MG_NONE: the coordinate) */
  MG_OP_UFAPP = 33,     /* a = argument, p0 = table, p1 = coord */
  MG_OP_KECCAK = 34,    /* a = data (or MG_NONE), p0 = byte length */
  MG_OP_EXP = 35,
  MG_OP_COUNT = 36
};

/* AUX: a generator-only scalar (no symbol of the query; e.g. one 256-bit calldata
 * word whose bytes are the lazy defaults of 32 calldata sites) */
enum mg_coord_kind { MG_COORD_SCALAR = 0, MG_COORD_ARRAY_SITE = 1, MG_COORD_UF_SITE = 2, MG_COORD_AUX = 3 };
enum mg_table_kind { MG_TABLE_ARRAY = 0, MG_TABLE_UF = 1 };

/* ---- candidate generator (search mode), format GEN3 -------------------- *
 * blob: header[4] {MG_GEN_MAGIC, n_coords, n_const_words, 0}
 *       specs: n_coords x 8 words {kind, p0, p1, p2, p3, p4, p5, p6}
 *       consts: n_const_words
 *
 * Coordinate c of candidate i is a pure function of (seed, i, c).  Two keys:
 *   fmix64(x)   = x ^= x>>33; x *= 0xFF51AFD7ED558CCD; x ^= x>>33;
 *                 x *= 0xC4CEB9FE1A85EC53; x ^= x>>33        (a bijection of u64)
 *   group key   G = fmix64((i >> 6) ^ fmix64(seed ^ 0xBB67AE8584CAA73B)) (G_lo, G_hi)
 *   lane key    K = G ^ fmix64((i & 63) ^ fmix64(seed ^ 0x6A09E667F3BCC908))  (K_lo, K_hi)
 * G is a bijection of the group number and K of the lane within a group, so the
 * pair (G, K) is distinct for every index (all 2^64 indices are usable).  G is
 * shared by the 64 consecutive indices of one aligned group — exactly one wave of
 * the search kernels — so a choice made from G is wave-uniform (a scalar branch,
 * not a per-lane select); the lane half of K is a per-thread constant.
 *   salt(c, j)  = c*0x9E3779B9 + j*0x85EBCA6B + 0x27D4EB2F           (mod 2^32)
 *   fin(x)      = x ^= x>>16; x = (x & 0xFFFFFF) * 0x9E3779; x ^= x>>15  (mod 2^32)
 *   rnd(c, j)   = fin(K_lo ^ salt(c, j)) + K_hi      per-lane 32 random bits
 *   h(c)        = rnd(c, 0xFFFF)                     per-lane index / delta bits
 *   wsel(c)     = (G_lo ^ salt(c, 0xFFFE)) * 0x9E3779B1 + G_hi   per-group choice bits
 *   raw uniform limbs u_0 = rnd(c, 0), u_1 = rnd(c, 1),
 *               u_j = lo32((u_{j-1} : u_{j-2}) >> s_j) + u_{j-2}  (mod 2^32, j >= 2),
 *               s_j = (7j + 3) mod 31 + 1
 *
 * Kinds (L = ceil(w/32) limbs; every value is masked to its width w):
 *   UNIFORM  limb j = u_j
 *   RANGE    lo + (((u64)rnd(c,0) * span) >> 32) (span 0: + rnd(c,0)), carried over L limbs
 *   DICT     entry ((h(c) >> 16) * n) >> 16 of the n-entry table
 *   ALIGNED  lo + (m << p1), m = ((u64)rnd(c,0) * count) >> 32 (count 0: m = rnd(c,0))
 *   FIXED    the value
 *   LAZY     never generated (a site whose default is a program node)
 *   MIXED    one alternative per aligned group, chosen by s = wsel(c) >> 16:
 *              pc = P(copy) if p3 != MG_NONE else 0, pd = P(dict) if n else 0, ps = P(small)
 *              s < pc            COPY     the FINAL value of coordinate p3 (p3 < c, same width)
 *              s < pc+pd         DICT     entry ((h(c) >> 16) * n) >> 16
 *              s < pc+pd+ps      SMALL    UNIFORM (u_j) masked to min(w, small_bits) bits
 *              otherwise         UNIFORM
 *            narrow coordinates (w <= MG_GEN_NARROW_BITS) take UNIFORM / SMALL from
 *            h(c) & 0xFFFF (one hash each);
 *            COPY and DICT add a per-lane delta when (wsel(c) & 0xFFFF) < P(delta):
 *              +/-(1 + (h & 1)), minus when (h >> 1) & 1, modulo 2^(32 L);
 *            then mask to w, then the clamp record (if any): v stays if
 *              lo <= v < lo + span, else v = lo + (((u64)limb0(v) * span) >> 32)
 *              (span 0 = 2^32; lo + span <= 2^w is checked at load).
 * Finally every kind applies its fixed-bit record (kind bits 8..31).
 * Probabilities are 16-bit fixed point (/65536).
 */
#define MG_GEN_MAGIC 0x334E4547u /* "GEN3" */
#define MG_GEN_NARROW_BITS 16u
#define MG_GEN_MAX_COPY_DEPTH 64u  /* longest static COPY chain a generator may hold */
enum mg_gen_kind {
  MG_GEN_UNIFORM = 0,  /* uniform over [0, 2^w) */
  MG_GEN_RANGE = 1,    /* p0 = const offset of lo, p1 = span (0 => 2^32): lo + r mod span */
  MG_GEN_DICT = 2,     /* p0 = const offset of n entries (ceil(w/32) limbs each), p1 = n */
  MG_GEN_MIXED = 3,    /* p0/p1 = dict, p2 = P(copy) | P(dict) << 16, p3 = copy-from coord (MG_NONE: none),
                          p4 = P(small) | small_bits << 16, p5 = P(delta on COPY/DICT),
                          p6 = 0 or 1 + const offset of a clamp record {lo limbs[L], span} */
  MG_GEN_ALIGNED = 4,  /* p0 = const offset of lo, p1 = log2(align), p2 = count (0 => 2^32) */
  MG_GEN_FIXED = 5,    /* p0 = const offset of the value */
  MG_GEN_LAZY = 6      /* site coords only: p0 = node whose value is the default (must precede the site) */
};

/* spec.kind bits 8..31: 0, or 1 + the const offset of a fixed-bit record
 * {mask limbs[L], value limbs[L]} (L = limbs of the coordinate) applied last:
 * v = (v & ~mask) | value. */
#define MG_GEN_KIND(kind) ((kind) & 0xFFu)

/* search flags */
#define MG_SEARCH_EARLY_EXIT 1u   /* stop lanes past the current first hit; skip waves whose roots all failed */
/* set by the engine itself (callers need not): the launch's first-hit word may be lowered by waves on
 * ANOTHER physical GPU (an in-process search split over devices), so kernels read it with system
 * scope (gfx950: global_load ... sc0 sc1) instead of agent scope (sc1) */
#define MG_SEARCH_SYSTEM_SCOPE 2u

typedef struct mg_program_info {
  uint32_t n_nodes, n_instrs, n_coords, n_roots;
  uint32_t value_words;      /* per-lane value-file words after liveness allocation */
  uint32_t uses_lds;         /* 1 if the value file lives in LDS */
  uint32_t n_watch;
  uint32_t watch_words;      /* sum of ceil(w/32) over watch nodes */
  uint32_t coord_words;      /* sum of ceil(w/32) over coords (SoA rows of mg_eval input) */
  uint32_t reserved;
  uint64_t limb_ops;         /* algorithmic 32-bit limb ops per candidate (fixed cost table) */
} mg_program_info_t;

typedef struct mg_stats {
  uint64_t programs_loaded;
  uint64_t launches;
  uint64_t candidates;       /* candidates evaluated (eval + search) */
  uint64_t hits;
  double kernel_ms_total;    /* HIP-event time of engine kernels on the engine stream */
  double last_kernel_ms;     /* HIP-event time of the last launch */
  uint64_t last_candidates;
  uint32_t device;
  uint32_t cu_count;
  uint32_t clock_mhz;
  uint32_t n_devices;  /* logical devices mg_init opened (the mask's GPUs) */
  uint64_t jit_refused;  /* JIT code objects the load gate refused (mg_code_object_check) */
} mg_stats_t;

/* device_mask: every set bit d opens GPU d (0 = GPU 0); all or nothing (a device that fails
 * to open closes the others and mg_init returns the error).  With several, mg_search and
 * mg_jit_search split a call of at least 2^20 candidates per device (MYTHGPU_SPLIT_MIN) over
 * them (mg_split_range: contiguous, group-aligned slices in index order), run the slices
 * concurrently, one stream per device, and reduce on the host (first hit = min, hits = sum);
 * smaller, latency-bound calls and every other call run on the first device.  Programs, generators and JIT kernels are mirrored under the same
 * handles and uploaded to a device on first use there. */
int mg_init(uint32_t device_mask);
/* the exchange step of a split search: 0 = host reduction (default), 1 = ONE RCCL all-reduce(min) of
 * the devices' first-hit words over xGMI (MYTHGPU_COLLECTIVE=rccl and a mask of distinct physical
 * GPUs; =rccl-force also on one device).  librccl is dlopen'ed; any failure keeps the host reduction. */
int mg_collective_kind(void);
/* host-only: the slice of [start, start+count) device d of n_dev sweeps */
int mg_split_range(uint64_t start, uint64_t count, uint32_t n_dev, uint64_t* starts, uint64_t* counts);
void mg_shutdown(void);
const char* mg_last_error(void);
int mg_version(void);

/* host-only checks (no GPU needed) */
int mg_program_check(const uint8_t* ssa, size_t len, mg_program_info_t* info);
/* ... and the program specialised for a generator blob (what mg_gen_info reports) */
int mg_program_check_gen(const uint8_t* ssa, size_t len, const uint32_t* gen_blob, size_t gen_words,
                         mg_program_info_t* info);

/* host-only: the lowered program a search (gen_blob) or an eval (gen_blob = NULL) actually
 * runs after specialisation, in SSA form, for inspection and for the oracle-side check that
 * specialisation keeps every verdict (tests/test_specialize_cpu.py).  Layout (uint32 words):
 * {MG_SPEC_MAGIC, n_instr, n_consts, n_aux, n_values, n_coords}, n_instr x 8-word
 * instructions {op, width, dst, a, b, c, p0, p1} (operands are value ids; op codes are the
 * device ops of mythril_amd/csrc/program.hpp), consts, aux (LOOKUP prior pairs), value
 * widths.  buf = NULL: only *out_words. */
#define MG_SPEC_MAGIC 0x43455053u /* "SPEC" */
#define MG_SPEC_KEEP_WATCH 1u
#define MG_SPEC_INTERP 2u     /* the interpreter's program (narrowed literal-tail keys), before slots */
int mg_program_specialized(const uint8_t* ssa, size_t len, const uint32_t* gen_blob, size_t gen_words,
                           uint32_t flags, uint32_t* buf, size_t cap_words, size_t* out_words);

int mg_program_load(const uint8_t* ssa, size_t len, uint64_t* prog_handle);
int mg_program_info(uint64_t prog, mg_program_info_t* info);
int mg_program_free(uint64_t prog);

/* a generator also specialises the program for the candidates it draws (range-decided
 * compares folded, dead code removed): mg_gen_info describes what searches run */
int mg_gen_load(uint64_t prog, const uint32_t* blob, size_t n_words, uint64_t* gen_handle);
int mg_gen_info(uint64_t gen, mg_program_info_t* info);
int mg_gen_free(uint64_t gen);

/* soa_coords: coord_words rows of n uint32 (row r = limb of a coordinate, coords in order)
 * verdict_out: n bytes (0/1); watch_out (nullable): watch_words rows of n uint32 */
int mg_eval(uint64_t prog, const uint32_t* soa_coords, uint64_t n, uint8_t* verdict_out, uint32_t* watch_out);
int mg_eval_dev(uint64_t prog, const uint32_t* d_soa_coords, uint64_t n, uint8_t* d_verdict_out,
                uint32_t* d_watch_out);
int mg_eval_generated(uint64_t prog, uint64_t gen, uint64_t seed, uint64_t start, uint64_t n,
                      uint8_t* verdict_out, uint32_t* watch_out);

/* first_hit: lowest satisfying candidate index in [start, start+count), UINT64_MAX if none.
 * assign_out (nullable): on a hit, the winning candidate's watch rows (program watch list,
 * watch_words uint32: the model read-back of Solver.model(), laser/smt/solver/solver.py:59-64) */
int mg_search(uint64_t prog, uint64_t gen, uint64_t seed, uint64_t start, uint64_t count, uint32_t flags,
              uint64_t* first_hit, uint64_t* n_hits, uint32_t* assign_out);

/* ---- JIT specialisation (comgr; hipRTC fallback) -----------------------
 * The compiler runs in a helper process (mythgpu_jitd, next to the library; started on the
 * first compile, MYTHGPU_JIT_ISOLATE=0 compiles in-process): a compiler abort fails that
 * compile with MG_E_UNSUPPORTED and turns the JIT off for the process; searches go on on
 * the interpreter.  mg_jit_helper_pid: its pid, -1 before the first compile, -2 after it died. */
int mg_jit_helper_pid(void);
/*
 * mg_jit_compile turns a loaded program into straight-line gfx950 code: with a
 * generator handle, the search kernel (mg_jit_search) specialised on it; with
 * gen = 0, the eval kernel (mg_jit_eval*).  It emits straight-line code (values in VGPRs, literals as immediates,
 * generator inlined).  Same semantics as mg_search / mg_eval. */
/* host-only: the specialised source (search kernel if gen_blob, else eval kernel); compile bit 0:
 * also compile it, bit 1: the eval kernel for the tiled SoA (MG_JIT_SOA_TILED).  Same bits for
 * mg_program_jit_asm. */
int mg_program_jit_source(const uint8_t* ssa, size_t len, const uint32_t* gen_blob, size_t gen_words, int compile,
                          char* buf, size_t cap, size_t* out_len);
/* host-only: the first tier's assembly (search + gen kernels with a generator blob, else the eval
 * kernel), optionally assembled */
int mg_program_jit_asm(const uint8_t* ssa, size_t len, const uint32_t* gen_blob, size_t gen_words, int compile,
                       char* buf, size_t cap, size_t* out_len);
/* host-only: the load gate every JIT code object passes before hipModuleLoadData (compiled or from
 * the disk cache).  It reads the AMDHSA kernel descriptors: *kernels, the largest private segment
 * per lane and LDS size over them, and whether any uses a dynamic stack (kernel_code_properties bit
 * 11).  Returns MG_OK if the object would load, MG_E_UNSUPPORTED if the gate refuses it (a dynamic
 * stack, more than MYTHGPU_JIT_PRIVATE_CAP bytes of private segment per lane — default 16 KiB — or
 * more than 160 KiB of LDS), MG_E_INVALID if it is not a code object.  Out pointers may be null.
 * A refused compile fails its JIT request with MG_E_UNSUPPORTED (search stays on the interpreter,
 * the get_model hook on z3); mg_stats counts refusals in jit_refused. */
int mg_code_object_check(const void* code, size_t len, uint32_t* kernels, uint32_t* max_private_bytes,
                         uint32_t* max_group_bytes, uint32_t* dynamic_stack);
int mg_jit_compile(uint64_t prog, uint64_t gen, uint64_t* jit_handle);
/* flags: MG_JIT_GEN_VERDICTS also builds mgj_gen (per-candidate verdicts, mg_jit_verdicts);
 * MG_JIT_ASM builds the first tier instead: the same kernels emitted as gfx950 assembly with the
 * engine's own register allocation, assembled and linked in a few ms (clang + LLVM take ~140 ms);
 * MG_E_UNSUPPORTED for the rare program outside it (too many live 256-bit values for the VGPRs).
 * An eval kernel WITH watch rows (model read-back, batched term evaluation) is the first tier's by
 * default — no SGPR spills by construction (the O3 kernel's row stores spill) — and the O3 kernel
 * only when the first tier refuses the program; MG_JIT_O3 asks for the O3 kernel (as does
 * MYTHGPU_JIT_WATCH_TIER=o3).  mg_jit_info's MG_JIT_ASM bit tells which one was built.
 * MG_JIT_SOA_TILED (eval kernel, gen = 0): the kernel reads a TILED SoA — coordinate limb row r of
 * candidate i at word ((i / 64) * coord_words + r) * 64 + i % 64, so a group of 64 candidates has
 * its rows in one contiguous block (coord_words * 256 bytes) — instead of [row][candidate].  The
 * buffer holds ceil(n / 64) whole blocks (the last one padded).  Same verdicts and watch rows. */
#define MG_JIT_GEN_VERDICTS 1u
#define MG_JIT_ASM 2u
#define MG_JIT_SOA_TILED 4u
#define MG_JIT_O3 8u
int mg_jit_compile_ex(uint64_t prog, uint64_t gen, uint32_t flags, uint64_t* jit_handle);
int mg_jit_verdicts(uint64_t jit, uint64_t seed, uint64_t start, uint64_t n, uint8_t* verdict_out);
/* Asynchronous compile on the engine's compile thread (outside the engine lock: searches on
 * the interpreter keep launching meanwhile).  mg_jit_poll: *jit_handle = 0 while pending
 * (wait_ms: 0 = do not wait, < 0 = wait until done); the ticket is consumed once it reports
 * a handle or an error.  mg_jit_cancel drops a ticket (a finished kernel is freed, a pending
 * one is discarded when it completes).  mg_jit_compile_ex = submit + wait. */
int mg_jit_compile_async(uint64_t prog, uint64_t gen, uint32_t flags, uint64_t* ticket);
int mg_jit_poll(uint64_t ticket, int32_t wait_ms, uint64_t* jit_handle);
int mg_jit_cancel(uint64_t ticket);
/* Drop the engine's host-side caches (lowered programs, generator specialisations, JIT code
 * objects by source): the next query pays every pass again (cold-start measurement). */
int mg_cache_clear(void);
int mg_jit_info(uint64_t jit, double* compile_ms, int* blocks_per_cu);
/* what a JIT handle was built as and the eval buffers it expects: *flags gets MG_JIT_ASM (the first
 * tier's kernels), MG_JIT_SOA_TILED (its eval kernel reads the tiled SoA) and MG_JIT_GEN_VERDICTS
 * (mgj_gen present); *coord_words / *watch_words the rows of the program's SoA and watch buffers, so
 * a caller of mg_jit_eval can check its buffers (coord_words x n, or coord_words x ceil(n/64) x 64
 * words when tiled).  Any out pointer may be null. */
int mg_jit_layout(uint64_t jit, uint32_t* flags, uint32_t* coord_words, uint32_t* watch_words);
int mg_jit_free(uint64_t jit);
int mg_jit_search(uint64_t jit, uint64_t seed, uint64_t start, uint64_t count, uint32_t flags, uint64_t* first_hit,
                  uint64_t* n_hits, uint32_t* assign_out);
/* n independent searches of one kernel (seed q over [starts[q], starts[q] + counts[q])), each
 * with its own hit buffer, launched back to back round-robin over four streams so one launch's
 * tail overlaps the next one's start, one wait for all: SURVEY's C2 sweep (2^24 per launch,
 * seeds 1..16) without a host round trip per launch.  first_hits[q] = ~0 when launch q found
 * nothing.  Results equal n calls of mg_jit_search; over several devices it is those calls. */
int mg_jit_search_many(uint64_t jit, uint32_t n, const uint64_t* seeds, const uint64_t* starts, const uint64_t* counts,
                       uint32_t flags, uint64_t* first_hits, uint64_t* n_hits);
int mg_jit_eval(uint64_t jit, const uint32_t* soa_coords, uint64_t n, uint8_t* verdict_out, uint32_t* watch_out);
int mg_jit_eval_dev(uint64_t jit, const uint32_t* d_soa_coords, uint64_t n, uint8_t* d_verdict_out,
                    uint32_t* d_watch_out);

/* msgs: concatenated messages; lens: n byte lengths; out32: n x 32 bytes */
int mg_keccak256(const uint8_t* msgs, const uint32_t* lens, uint64_t n, uint8_t* out32);

int mg_stats(mg_stats_t* out);
int mg_stats_reset(void);

/* device buffer helpers for callers that keep inputs resident in HBM */
int mg_dev_alloc(size_t bytes, void** dptr);
int mg_dev_free(void* dptr);
int mg_dev_upload(void* dptr, const void* src, size_t bytes);
int mg_dev_download(void* dst, const void* dptr, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* MYTHGPU_H */
