"""The first JIT tier (``mythril_amd/csrc/jit_asm.cpp``) against the C port on the CPU, at depth.

``tests/asmsim/`` is an instruction-level simulator of the gfx950 subset the tier emits: it runs
``mgj_gen``, ``mgj_search`` and ``mgj_eval`` wave by wave and also checks the emitter's own
claims — no register read while a load into it is in flight (vmcnt / lgkmcnt), the VALU->SGPR->VALU
and VALU->SGPR->VMEM wait states, the constant-bus and literal rules, every access inside a
buffer or the kernel's LDS, no read of a never-written VGPR.  The driver (``asmsim_main.cpp``)
emits the kernels exactly as ``mg_jit_compile_ex`` does and compares, per record:

* ``mgj_gen`` verdicts per candidate with the C port's (``oracle/bveval.c``, the unspecialised
  program) on a random 63-bit window; ``mgj_search``'s first hit and hit count; the early-exit
  first hit, and that the hit was also lowered into a peer device's hit word;
* ``mgj_eval`` verdicts (row-major and tiled SoA) on random coordinate rows.

The emitter and the specialiser run under AddressSanitizer + UndefinedBehaviorSanitizer (g++;
the simulator and the C port, test infrastructure, at -O2).  Programs: ``MYTHGPU_SIMFUZZ_N``
(default 10,000) LASER-shaped queries (``tests/lasergen.py``: dispatchers, actor sets, keccak-keyed
mappings with many-prior inverse lookups and literal-slot tails, Store chains, wrap predicates, ITE
guards, symbol equalities that make MIXED coordinates copy each other in chains), split over four
emitter configurations (the lookup-compare pushdown and the guarded-lookup pruning on and off, the
difference cache, Bool lookups, limb-pair dictionary reads, index compares and NOT folding off, no
literal pool with the LDS-staged eval row queue), plus
random programs over the tier's
operators and the workloads at several windows.

Reference anchor: a candidate's verdict is ``Model.eval(And(constraints), model_completion=True)``
(``mythril/laser/smt/model.py:45-59``) of the query ``get_model`` receives
(``mythril/support/model.py:15-49``).
"""
import multiprocessing as mp
import os
import random
import shutil
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
N_FUZZ = int(os.environ.get("MYTHGPU_SIMFUZZ_N", "10000"))
WORKERS = max(1, min(8, os.cpu_count() or 1))
CONFIGS = [
    {},
    {"MYTHGPU_EQ_PUSHDOWN": "0", "MYTHGPU_ITE_PRUNE": "0"},
    {"MYTHGPU_JIT_ASM_NO_EQ_CACHE": "1", "MYTHGPU_JIT_ASM_NO_BOOL_LOOKUP": "1", "MYTHGPU_JIT_ASM_EXIT_SKIP": "0",
     "MYTHGPU_JIT_ASM_LDS_B32": "1", "MYTHGPU_JIT_ASM_NO_DICT_EQ": "1", "MYTHGPU_FOLD_NOT": "0",
     "MYTHGPU_JIT_ASM_NO_KFOLD": "1", "MYTHGPU_JIT_ASM_NO_MULHI24": "1", "MYTHGPU_JIT_ASM_ALIGNED_MAD": "0"},
    {"MYTHGPU_JIT_ASM_NOPOOL": "1", "MYTHGPU_EQ_PUSHDOWN": "1", "MYTHGPU_JIT_ASM_GLDS": "1"},
]


def _build(out: Path, sanitize: bool) -> Path:
    from mythril_amd import build

    build.write_prelude()
    cxx, cc = shutil.which("g++"), shutil.which("gcc")
    if cxx is None or cc is None:
        pytest.skip("g++/gcc not available")
    out.mkdir(parents=True, exist_ok=True)
    san = ["-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer"] if sanitize else ["-O2"]
    jobs = []
    objs = []
    # the product's emitter and specialiser (under the sanitizers), the checker and the simulator
    for src, flags, lang in [
        ("mythril_amd/csrc/program.cpp", san, cxx), ("mythril_amd/csrc/jit_asm.cpp", san, cxx),
        ("tests/asmsim/asmsim_main.cpp", san, cxx), ("tests/asmsim/asmsim.cpp", ["-O2"], cxx),
        ("oracle/bveval.c", ["-O2"], cc),
    ] + ([] if sanitize else [("mythril_amd/csrc/jit.cpp", ["-O2"], cxx)]):
        o = out / (Path(src).name + ".o")
        cmd = [lang] + (["-std=c++17"] if lang == cxx else []) + flags + [
            "-I/opt/rocm/include", f"-I{ROOT}", "-c", str(ROOT / src), "-o", str(o)]
        if not sanitize:
            cmd.append("-DASMSIM_ASSEMBLER")
        jobs.append(subprocess.Popen(cmd, stderr=subprocess.PIPE, text=True))
        objs.append(str(o))
    for j in jobs:
        _, e = j.communicate(timeout=900)
        assert j.returncode == 0, e[-3000:]
    exe = out / ("asmsim_asan" if sanitize else "asmsim")
    r = subprocess.run([cxx] + san + objs + ["-ldl", "-o", str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


SOURCES = ["mythril_amd/csrc/program.cpp", "mythril_amd/csrc/program.hpp", "mythril_amd/csrc/jit_asm.cpp",
           "mythril_amd/csrc/jit.hpp", "include/mythgpu.h", "tests/asmsim/asmsim_main.cpp", "tests/asmsim/asmsim.cpp",
           "tests/asmsim/asmsim.hpp", "oracle/bveval.c"]


def _cached(tmp_path_factory, sanitize: bool) -> Path:
    """A driver build, cached under /tmp by a hash of its sources (a rebuild costs ~40 s)."""
    import hashlib

    h = hashlib.sha256()
    for s in SOURCES + (["mythril_amd/csrc/jit.cpp"] if not sanitize else []):
        h.update((ROOT / s).read_bytes())
    cache = Path("/tmp") / f"mythgpu-asmsim-{h.hexdigest()[:16]}"
    name = "asmsim_asan" if sanitize else "asmsim"
    exe = cache / name
    if exe.exists():
        return exe
    built = _build(tmp_path_factory.mktemp(name), sanitize=sanitize)
    cache.mkdir(parents=True, exist_ok=True)
    shutil.copy2(built, cache / (name + ".tmp"))
    os.replace(cache / (name + ".tmp"), exe)
    return exe


@pytest.fixture(scope="module")
def sim(tmp_path_factory):
    """The differential driver (emitter, simulator and C port at -O2; comgr's assembler linked)."""
    return _cached(tmp_path_factory, sanitize=False)


@pytest.fixture(scope="module")
def sim_asan(tmp_path_factory):
    """The emitter and the specialiser under ASan + UBSan (run with ASMSIM_EMIT_ONLY=1)."""
    return _cached(tmp_path_factory, sanitize=True)


def record(kind, pb: bytes, blob, seed: int, start: int, count: int, flags: int = 0) -> bytes:
    out = struct.pack("<II", kind, len(pb)) + pb
    if blob is None:
        out += struct.pack("<I", 0xFFFFFFFF)
    else:
        g = np.asarray(blob, dtype=np.uint32)
        out += struct.pack("<I", len(g)) + g.tobytes()
    return out + struct.pack("<QQII", seed, start, count, flags)


def run_sim(exe: Path, records: bytes, env_extra=None, timeout=1500):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    env.update(env_extra or {})
    r = subprocess.run([str(exe)], input=records, capture_output=True, env=env, timeout=timeout)
    out = r.stdout.decode(errors="replace")
    err = r.stderr.decode(errors="replace")
    lines = out.strip().splitlines()
    summary = dict(kv.split("=") for kv in lines[-1].split()) if lines and "records=" in lines[-1] else {}
    return r.returncode, summary, lines[:-1], err


def _fuzz_records(lo: int, hi: int, full: bool = False) -> bytes:
    """LASER-shaped queries ``lo .. hi`` as search records (``full``: with symbolic division,
    signed division / remainder, variable shifts, EXP and concrete Keccak)."""
    from mythril_amd import search
    from tests.lasergen import laser_query

    recs = []
    for s in range(lo, hi):
        roots = laser_query(s + (500_000 if full else 0), full=full)
        P, blob = search.prepare(roots)
        rng = random.Random(s * 7919 + 1)
        start = rng.getrandbits(63)
        if s % 3 == 0:
            start = (start & ~0xFFFFFFFF) | 0x80000000 | rng.getrandbits(31)  # bit 31 of the low word set
        if s % 5 == 0:
            start = rng.getrandbits(12)  # from near index 0 (the product's early-exit shape)
        # every 25th kernel also goes through comgr's assembler and linker (encodings, operand rules)
        recs.append(record(0, P.to_bytes(), blob, rng.getrandbits(32), start, 640 if s % 10 == 0 else 256,
                           flags=int(s % 25 == 0)))
    return b"".join(recs)


def _fuzz_worker(args):
    exe, asan, lo, hi, cfg = args
    recs = _fuzz_records(lo, hi)
    env = dict(CONFIGS[cfg], MYTHGPU_JIT_ASM_CHECK="1")
    out = []
    for e, extra in ((asan, {"ASMSIM_EMIT_ONLY": "1"}), (exe, {})):
        rc, summary, bad, err = run_sim(Path(e), recs, dict(env, **extra))
        out.append((rc, summary, bad[:5], err[-3000:], cfg))
    return out


def _check(results, n_expected):
    total = {"records": 0, "ok": 0, "outside": 0}
    for rc, summary, bad, err, cfg in results:
        assert summary, f"config {CONFIGS[cfg]}: no summary (rc {rc})\n{err}"
        assert rc == 0 and "Sanitizer" not in err and "runtime error" not in err, \
            f"config {CONFIGS[cfg]}: {summary}\n" + "\n".join(bad) + "\n" + err
        for k in total:
            total[k] += int(summary[k])
    assert total["records"] == n_expected
    return total


def test_asm_tier_laser_fuzz_under_asan(sim, sim_asan):
    """>= 10,000 LASER-shaped queries: every first-tier verdict, first hit and hit count equals the
    C port's, with no simulator rule broken, no lifetime violation from the emitter's own checker
    (MYTHGPU_JIT_ASM_CHECK) and no sanitizer report from the emitter and the specialiser."""
    n = N_FUZZ
    step = max(1, n // (WORKERS * 4))
    tasks = [(str(sim), str(sim_asan), lo, min(n, lo + step), (lo // step) % len(CONFIGS))
             for lo in range(0, n, step)]
    with mp.get_context("fork").Pool(WORKERS) as pool:
        results = pool.map(_fuzz_worker, tasks, chunksize=1)
    asan_total = _check([r[0] for r in results], n)
    total = _check([r[1] for r in results], n)
    print("laser fuzz:", total, "emitter under ASan:", asan_total)
    # the queries are LASER's vocabulary, inside the tier by construction
    assert total["ok"] == n and asan_total["ok"] == n, (total, asan_total)


def _tier_records(lo, hi, full=False) -> bytes:
    """Random programs over the tier's operators as search + eval records."""
    from mythril_amd import search
    from tests.helpers import random_tier_program

    recs = []
    for s in range(lo, hi):
        roots = random_tier_program(10_000 + s + (500_000 if full else 0), full=full)
        P, blob = search.prepare(roots)
        rng = random.Random(s)
        recs.append(record(0, P.to_bytes(), blob, rng.getrandbits(32), rng.getrandbits(63), 192))
        # the eval kernel on the same program (watch list off: verdict rows only)
        prev = P.watch
        P.set_watch([])
        pb = P.to_bytes()
        P.set_watch(prev)
        recs.append(record(1 + (s & 1), pb, None, rng.getrandbits(32), 0, 64 * rng.randint(1, 5) + rng.randrange(64)))
    return b"".join(recs)


def _tier_worker(args):
    exe, lo, hi, cfg = args
    rc, summary, bad, err = run_sim(Path(exe), _tier_records(lo, hi), dict(CONFIGS[cfg], MYTHGPU_JIT_ASM_CHECK="1"))
    return rc, summary, bad[:5], err[-3000:], cfg


def test_asm_tier_random_programs_sim(sim):
    """Random programs over the tier's operators (every width from 8 to 512, ITE, Extract/Concat,
    Zero/SignExt, array Select/Store, UF applications, bvumul_noovfl): search, gen and eval
    kernels against the C port."""
    n = int(os.environ.get("MYTHGPU_SIMFUZZ_TIER_N", "1000"))
    step = max(1, n // (WORKERS * 2))
    tasks = [(str(sim), lo, min(n, lo + step), (lo // step) % len(CONFIGS)) for lo in range(0, n, step)]
    with mp.get_context("fork").Pool(WORKERS) as pool:
        results = pool.map(_tier_worker, tasks, chunksize=1)
    total = _check(results, 2 * n)
    print("tier programs:", total)
    assert total["ok"] >= 2 * n * 0.9, total


def test_asm_tier_workloads_sim(sim):
    """The workloads inside the tier and the bench's hard needle: search/gen at windows with bit 31
    of the low word set and from index 0, and the eval kernel (row-major and tiled) over several
    64-candidate groups per wave (the cross-group row ring)."""
    import bench
    from mythril_amd import search, workloads

    recs = []
    queries = {n: [c.raw for c in workloads.WORKLOADS[n]()] for n in workloads.WORKLOADS}
    queries["hard_needle"] = bench.hard_query(workloads.WORKLOADS["token_transfer_underflow"]())
    rng = random.Random(5)
    n_search = 0
    for name, roots in sorted(queries.items()):
        P, blob = search.prepare(roots)
        pb = P.to_bytes()
        for start in (0, 0x80000001 | (rng.getrandbits(30) << 33), rng.getrandbits(63)):
            recs.append(record(0, pb, blob, rng.getrandbits(32), start, 4096))
            n_search += 1
        prev = P.watch
        P.set_watch([])
        pe = P.to_bytes()
        P.set_watch(prev)
        for kind in (1, 2):
            recs.append(record(kind, pe, None, rng.getrandbits(32), 0, 64 * 9 + 37))
    rc, summary, bad, err = run_sim(sim, b"".join(recs), {"MYTHGPU_JIT_ASM_CHECK": "1"})
    assert rc == 0, f"{summary}\n" + "\n".join(bad) + "\n" + err[-3000:]
    # sha3_keyed_mapping (Keccak, EXP, SDIV) is the one workload outside the tier today
    assert int(summary["ok"]) + int(summary["outside"]) == len(recs)
    assert int(summary["ok"]) >= len(recs) - 5


def test_asm_signed_literal_compares_and_views_sim(sim):
    """Signed compares against literals (the sign test + high-limb equality path) at every shape of
    literal — zero, small, at 2^31, multi-limb, -1, small negative, the extremes — on both sides,
    over operands whose high limbs are sign or zero extensions (so the high-limb equality is often
    true), and byte CONCAT chains read through by EXTRACTs and CONCATs (views): eval (row-major and
    tiled) and search kernels against the C port."""
    from mythril_amd import search
    from mythril_amd.smt import terms as T

    rng = random.Random(11)
    recs = []
    for w in (40, 64, 72, 96, 160, 256):
        x = T.BitVecVar(f"sx{w}", w)
        n8 = T.BitVecVar(f"n8_{w}", 8)
        n32 = T.BitVecVar(f"n32_{w}", 32)
        ops = [x, T.sign_extend(w - 8, n8), T.sign_extend(w - 32, n32), T.zero_extend(w - 32, n32)]
        lits = {0, 1, 29, (1 << 31) - 1, 1 << 31, (1 << 32) + 5, (1 << (w - 1)) - 1, 1 << (w - 1),
                (1 << w) - 1, (1 << w) - 2, (1 << w) - (1 << 33), (1 << w) - 200, (1 << w) - (1 << 31)}
        for k in sorted(lits):
            K = T.BitVecVal(k % (1 << w), w)
            for op in ("bvslt", "bvsle", "bvsgt", "bvsge"):
                a = rng.choice(ops)
                c1, c2 = T.bvcmp(op, a, K), T.bvcmp(op, K, rng.choice(ops))
                roots = [T.or_(c1, T.not_(c2)) if rng.random() < 0.5 else c1]
                P, blob = search.prepare(roots)
                recs.append(record(0, P.to_bytes(), blob, rng.getrandbits(32), rng.getrandbits(63), 128))
                prev = P.watch
                P.set_watch([])
                pe = P.to_bytes()
                P.set_watch(prev)
                recs.append(record(1 + (k & 1), pe, None, rng.getrandbits(32), 0, 64 * 3 + 5))
    # one value against many literals (the 32-bit clamp path): a sum of random weights over the compares
    # that hold, its low bits tested, so a single wrong compare changes the verdict more often than not
    for w in (40, 64, 96, 256):
        n8, n32 = T.BitVecVar(f"m8_{w}", 8), T.BitVecVar(f"m32_{w}", 32)
        for x in (T.BitVecVar(f"mx{w}", w), T.sign_extend(w - 8, n8), T.sign_extend(w - 32, n32),
                  T.zero_extend(w - 32, n32)):
            cs = []
            for k in (0, 1, 2, 3, 5, 29, 127, 128, 255, 1 << 31, 0xFFFFFFFE, 0xFFFFFFFF, 1 << 32, 1 << 38):
                K = T.BitVecVal(k % (1 << w), w)
                cs += [T.bvcmp("bvslt", K, x), T.bvcmp("bvslt", x, K), T.bvcmp("bvsle", x, K), T.bvcmp("bvsge", x, K)]
            acc = T.BitVecVal(0, 32)
            for c in cs:
                acc = T.bvbin("bvadd", acc, T.ite(c, T.BitVecVal(rng.getrandbits(32), 32), T.BitVecVal(0, 32)))
            P, blob = search.prepare([T.eq(T.extract(2, 0, acc), T.BitVecVal(rng.randrange(8), 3))])
            recs.append(record(0, P.to_bytes(), blob, rng.getrandbits(32), rng.getrandbits(63), 128))
            P.set_watch([])
            for kind in (1, 2):
                recs.append(record(kind, P.to_bytes(), None, rng.getrandbits(32), 0, 64 * 4 + 9))
    # an overflow check and the product it guards (batchOverflow): the MUL takes the UMUL_NOOVF's limbs
    for w in (64, 96, 256):
        for nb in (8, 32, w):
            cnt = T.zero_extend(w - nb, T.BitVecVar(f"c{w}_{nb}", nb)) if nb < w else T.BitVecVar(f"c{w}", w)
            val = T.BitVecVar(f"v{w}_{nb}", w)
            prod = T.bvbin("bvmul", cnt, val)
            for lo in (0, 3, w - 9):
                roots = [T.or_(T.not_(T.bvcmp("bvumul_noovfl", cnt, val)),
                               T.eq(T.extract(lo + 7, lo, prod), T.BitVecVal(rng.getrandbits(8), 8)),
                               T.bvcmp("bvult", prod, T.BitVecVal(rng.getrandbits(w - 2), w)))]
                P, blob = search.prepare(roots)
                recs.append(record(0, P.to_bytes(), blob, rng.getrandbits(32), rng.getrandbits(63), 128))
                P.set_watch([])
                recs.append(record(1 + (lo & 1), P.to_bytes(), None, rng.getrandbits(32), 0, 64 * 2 + 9))
    # byte chains: a word built from 32 bytes, read through by extracts and a wider concat
    bs = [T.BitVecVar(f"cb{i}", 8) for i in range(32)]
    word = bs[0]
    for b in bs[1:]:
        word = T.concat(word, b)
    for lo, hi in ((0, 255), (8, 263 - 8), (3, 40), (100, 131), (248, 255)):
        ex = T.extract(hi, lo, word)
        wide = T.concat(T.BitVecVar("cw", 24), T.concat(ex, T.BitVecVal(5, 8)))
        roots = [T.or_(T.bvcmp("bvult", T.extract(hi - lo, 0, wide), T.BitVecVal(1 << min(hi - lo, 200), hi - lo + 1)),
                       T.eq(T.extract(7, 0, wide), T.BitVecVal(5, 8)))]
        roots.append(T.not_(T.eq(T.extract(hi - lo + 8, 8, wide), T.BitVecVal(0, hi - lo + 1))))
        P, blob = search.prepare(roots)
        recs.append(record(0, P.to_bytes(), blob, rng.getrandbits(32), rng.getrandbits(63), 192))
        P.set_watch([])
        for kind in (1, 2):
            recs.append(record(kind, P.to_bytes(), None, rng.getrandbits(32), 0, 64 * 4 + 9))
    rc, summary, bad, err = run_sim(sim, b"".join(recs), {"MYTHGPU_JIT_ASM_CHECK": "1"})
    assert rc == 0, f"{summary}\n" + "\n".join(bad) + "\n" + err[-3000:]
    assert int(summary["ok"]) == len(recs), summary
    print("signed literal compares / views:", summary)


def test_asm_eval_spills_sim(sim, monkeypatch):
    """Eval kernels that spill values to LDS (Gen::spill_one / reload): random tier programs, the
    workloads and a many-key array read (canonicalising LOOKUPs over 64-bit keys, so keys collide)
    under an artificial 72-register file (MYTHGPU_JIT_ASM_SPILL_TEST), verdicts against the C port
    with the simulator's LDS, wait-count and lifetime checks; a kernel the spiller cannot fit is
    refused (the O3 kernel then), never wrong."""
    from mythril_amd import native, search, workloads
    from mythril_amd.smt import terms as T
    from tests.helpers import random_tier_program

    progs = []
    for s_ in range(80):
        P, _ = search.prepare(random_tier_program(30_000 + s_, full=bool(s_ & 1)))
        P.set_watch([])
        progs.append((P.to_bytes(), 1 + (s_ & 1)))
    for name in ("walletlibrary_kill", "token_transfer_underflow", "etherstore_reentrancy"):
        P, _ = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
        P.set_watch([])
        progs += [(P.to_bytes(), 1), (P.to_bytes(), 2)]
    arr = T.ArrayVar("Cd", 64, 8)
    keys = [T.BitVecVar(f"k{i}", 64) for i in range(48)]
    acc = T.BitVecVal(0, 32)
    rng = random.Random(3)
    for k in keys:
        acc = T.bvbin("bvadd", acc, T.bvbin("bvmul", T.zero_extend(24, T.select(arr, k)), T.BitVecVal(rng.getrandbits(32), 32)))
    P, _ = search.prepare([T.eq(T.extract(2, 0, acc), T.BitVecVal(5, 3))])
    P.set_watch([])
    progs += [(P.to_bytes(), 1), (P.to_bytes(), 2)]
    monkeypatch.setenv("MYTHGPU_JIT_ASM_SPILL_TEST", "72")
    spilled = 0
    for pb, kind in progs:
        try:
            spilled += native.jit_asm(pb, None, tiled=kind == 2).count("ds_write_b32") > 0
        except native.EngineUnsupported:
            pass
    recs = [record(kind, pb, None, rng.getrandbits(32), 0, 64 * rng.randint(1, 3) + rng.randrange(64)) for pb, kind in progs]
    rc, summary, bad, err = run_sim(sim, b"".join(recs), {"MYTHGPU_JIT_ASM_CHECK": "1", "MYTHGPU_JIT_ASM_SPILL_TEST": "72"})
    assert rc == 0 and summary, err[-3000:]
    assert summary["mismatch"] == "0" and summary["simerror"] == "0" and summary["asmerror"] == "0", (summary, bad[:5])
    assert int(summary["ok"]) >= len(recs) // 2 and spilled >= 5, (summary, spilled)
    print("spills:", summary, "kernels with spills:", spilled)


def _vmtest_readbacks(names=None, every=1):
    """VMTests model read-backs as eval programs (watch rows kept), the shape
    ``test_jit_vmtests_literals_as_runtime_inputs`` runs on the GPU: post-state storage words with
    every PUSH literal lifted into a runtime coordinate
    (``tests/laser/evm_testsuite/evm_test.py:109-188``)."""
    from mythril_amd import ssa
    from mythril_amd.smt import terms as T
    from tests.helpers import lift_literals, vmtest_cases

    out = []
    for ci, (name, v, r) in enumerate(vmtest_cases()):
        keys = [int(k, 16) for k in v["post_storage"]]
        if not keys or (names is not None and name not in names) or (names is None and ci % every):
            continue
        lifted, _ = lift_literals([r.storage_word(k).raw for k in keys])
        P = ssa.flatten([T.BoolVal(True)], extra=lifted)
        P.set_watch([P.term_node[w.id] for w in lifted])
        out.append((name, P.to_bytes()))
    return out


READBACK_SOLO = ("TestNameRegistrator", "expXY", "expXY_success")


def test_asm_eval_readbacks_sim(sim):
    """Model read-back kernels (watch rows stored) against the C port's values row by row — every
    eleventh VMTests read-back plus the three whose 63 live 256-bit calldata keys need more LDS
    spill slots than four waves of a workgroup can hold (160 KiB): those run `solo`, one working
    wave per workgroup with up to 639 lane-major slots and one 64-candidate group per workgroup, no
    group loop (jit_asm.cpp, Gen::solo), assembled and linked by comgr as well.  Until round 6 they
    went to the O3 tier (20-160 s of LLVM each)."""
    from mythril_amd import native

    progs = _vmtest_readbacks(every=11) + _vmtest_readbacks(names=READBACK_SOLO)
    assert len(progs) >= 30
    solo = 0
    for name, pb in progs:
        # inside the tier (no EngineUnsupported); the solo kernels also through comgr's assembler and
        # linker and the load gate (a 58 k-instruction kernel: no branch may span it)
        src = native.jit_asm(pb, None, compile=name in READBACK_SOLO)
        if name in READBACK_SOLO:
            assert "mgj_meta_eval_cpb:" in src and "ds_write_b32" in src, name
            lds = int(src.split(".amdhsa_group_segment_fixed_size ")[1].split()[0])
            assert 160 * 256 < lds <= 160 * 1024, (name, lds)  # past four waves' share, inside the CU's LDS
            solo += 1
    assert solo == 3
    rng = random.Random(17)
    recs = [record(1 + (i & 1), pb, None, rng.getrandbits(32), 0, 64 * 2 + 5, flags=int(name in READBACK_SOLO))
            for i, (name, pb) in enumerate(progs)]
    rc, summary, bad, err = run_sim(sim, b"".join(recs), {"MYTHGPU_JIT_ASM_CHECK": "1"})
    assert rc == 0 and summary, f"{summary}\n" + "\n".join(bad[:5]) + "\n" + err[-3000:]
    assert int(summary["ok"]) == len(recs), (summary, bad[:5])
    print("read-backs:", summary)


def _full_worker(args):
    exe, lo, hi, cfg, kind = args
    recs = _fuzz_records(lo, hi, full=True) if kind == "laser" else _tier_records(lo, hi, full=True)
    rc, summary, bad, err = run_sim(Path(exe), recs, dict(CONFIGS[cfg], MYTHGPU_JIT_ASM_CHECK="1"))
    return rc, summary, bad[:5], err[-3000:], cfg


def test_asm_tier_full_vocabulary_sim(sim):
    """Round 5's vocabulary in the tier — symbolic UDIV/UREM, SDIV/SREM/SMOD, variable SHL/LSHR/ASHR,
    EXP and Keccak-256 (one and several blocks) — per candidate equal to the C port on LASER-shaped
    queries (``lasergen.laser_query(full=True)``) and random programs (search, gen and eval kernels)."""
    n_l = int(os.environ.get("MYTHGPU_SIMFUZZ_FULL_N", "1000"))
    n_t = n_l // 2
    tasks = []
    step = max(1, n_l // (WORKERS * 2))
    tasks += [(str(sim), lo, min(n_l, lo + step), (lo // step) % len(CONFIGS), "laser") for lo in range(0, n_l, step)]
    step = max(1, n_t // WORKERS)
    tasks += [(str(sim), lo, min(n_t, lo + step), (lo // step) % len(CONFIGS), "tier") for lo in range(0, n_t, step)]
    with mp.get_context("fork").Pool(WORKERS) as pool:
        results = pool.map(_full_worker, tasks, chunksize=1)
    total = _check(results, n_l + 2 * n_t)
    print("full vocabulary:", total)
    # a refusal is a fall-back (the interpreter keeps the query), never a wrong verdict; one
    # program in ~2,000 keeps too many 256-bit values live around an EXP or Keccak (out of VGPRs)
    assert total["ok"] >= 0.995 * (n_l + 2 * n_t), total


def _mutants(tmp_path: Path, mutants) -> dict:
    """Drivers built with textual edits {name: {file: (old, new)}} of their sources (no sanitizers);
    the unedited objects are compiled once and shared, everything in parallel."""
    srcs = ("mythril_amd/csrc/program.cpp", "mythril_amd/csrc/jit_asm.cpp", "tests/asmsim/asmsim_main.cpp",
            "tests/asmsim/asmsim.cpp", "oracle/bveval.c")
    jobs, objs = [], {}

    def compile_(path: Path, o: Path, src: str):
        lang = ["gcc"] if src.endswith(".c") else ["g++", "-std=c++17"]
        jobs.append(subprocess.Popen(lang + ["-O1", f"-I{ROOT}", f"-I{ROOT / Path(src).parent}", "-I/opt/rocm/include",
                                             "-c", str(path), "-o", str(o)], stderr=subprocess.PIPE, text=True))

    for src in srcs:
        if any(src not in e for e in mutants.values()):
            o = tmp_path / f"base_{Path(src).name}.o"
            compile_(ROOT / src, o, src)
            objs[src] = o
    per = {}
    for name, edits in mutants.items():
        per[name] = []
        for src in srcs:
            if src not in edits:
                continue
            text = (ROOT / src).read_text()
            old, new = edits[src]
            assert old in text, (src, old)
            path = tmp_path / f"{name}_{Path(src).name}"
            path.write_text(text.replace(old, new))
            o = tmp_path / f"{name}_{Path(src).name}.o"
            compile_(path, o, src)
            per[name].append((src, o))
    for j in jobs:
        _, e = j.communicate(timeout=900)
        assert j.returncode == 0, e[-2000:]
    out = {}
    for name, own in per.items():
        mine = dict(objs)
        mine.update(dict(own))
        exe = tmp_path / name
        subprocess.run(["g++"] + [str(mine[s]) for s in srcs] + ["-ldl", "-o", str(exe)], check=True)
        out[name] = exe
    return out


def test_the_checks_have_teeth(sim, tmp_path):
    """The differential catches what it is for.  (1) An emitter with round 4's COPY-liveness bug put
    back (a MIXED coordinate's COPY branch reusing a copy source the depth-first order had already
    released; it gave false SATs on etherstore on the GPU) fails on etherstore.  (2) A simulator
    whose subtract-with-borrow is wrong reports mismatches: the emitter and the simulator do not
    merely agree with themselves."""
    from mythril_amd import search, workloads

    def recs(name, n=4, count=4096):
        P, blob = search.prepare([c.raw for c in workloads.WORKLOADS[name]()])
        rng = random.Random(1)
        return b"".join(record(0, P.to_bytes(), blob, rng.getrandbits(32), rng.getrandbits(63), count)
                        for _ in range(n))

    eth = recs("etherstore_reentrancy")
    rc, good, _, _ = run_sim(sim, eth, {"MYTHGPU_JIT_ASM_CHECK": "1"})
    assert rc == 0 and int(good["mismatch"]) == 0, good
    exes = _mutants(tmp_path, {
        "copy_bug": {"mythril_amd/csrc/jit_asm.cpp": ("if (it != cval.end() && val[it->second].def &&",
                                                      "if (it != cval.end() &&")},
        "sub_bug": {"tests/asmsim/asmsim.cpp": ("d[l] = (uint32_t)(u - b);", "d[l] = (uint32_t)(u - b + 1);")},
    })
    rc, summary, lines, _ = run_sim(exes["copy_bug"], eth)
    assert rc != 0 and int(summary["mismatch"]) > 0, (summary, lines)
    mixed = recs("token_transfer_underflow", 1, 1024) + recs("walletlibrary_kill", 1, 1024) + \
        recs("bectoken_batch_overflow", 1, 1024)
    rc, summary, lines, _ = run_sim(exes["sub_bug"], mixed)
    assert rc != 0 and int(summary["mismatch"]) > 0, (summary, lines)
