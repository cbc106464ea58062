"""Sanitizer fuzz of the library's untrusted-input parsers (CPU only, no GPU).

tests/fuzz/fuzz_host.cpp links program.cpp (lower_program, parse_gen,
specialize_program) and jit.cpp (jit_source) with g++ -fsanitize=address,undefined
-fno-sanitize-recover=all.  Hypothesis mutates valid program and GEN3 generator blobs
(the workloads' and random DAGs'; word-level: bit flips, boundary values, truncation,
extension, splices) and every mutant goes through the same calls mg_program_check_gen
and mg_jit_compile_ex make before any device work.  Pass = the process exits 0 with no
sanitizer report, and the seeds themselves are accepted.
"""
import os
import shutil
import struct
import subprocess
from pathlib import Path

import numpy as np
import pytest

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402

from helpers import RandomProgram  # noqa: E402
from mythril_amd import search, ssa, workloads  # noqa: E402

ROOT = Path(__file__).resolve().parent.parent
N_MUTANTS = int(os.environ.get("MYTHGPU_FUZZ_N", "10000"))
BOUNDARY = [0, 1, 2, 3, 7, 8, 31, 32, 33, 63, 64, 255, 256, 257, 512, 1024, 0xFFFF, 0x10000, 0x7FFFFFFF,
            0x80000000, 0xFFFFFFFE, 0xFFFFFFFF]


@pytest.fixture(scope="module")
def fuzz_bin(tmp_path_factory):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    from mythril_amd import build

    build.write_prelude()
    out = tmp_path_factory.mktemp("fuzz") / "fuzz_host"
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", f"-I{ROOT}", "-I/opt/rocm/include", str(ROOT / "tests/fuzz/fuzz_host.cpp"),
           str(ROOT / "mythril_amd/csrc/program.cpp"), str(ROOT / "mythril_amd/csrc/jit.cpp"), "-ldl", "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return out


def _seeds():
    seeds = []
    for name in sorted(workloads.WORKLOADS):
        roots = [c.raw for c in workloads.WORKLOADS[name]()]
        for aux in (False, True):
            P = ssa.flatten(roots, aux_words=aux)
            seeds.append((P.to_bytes(), search.default_generator(P, roots=roots).blob()))
    for s in range(6):
        rp = RandomProgram(s, n_ops=30)
        P = ssa.flatten([rp.root], extra=rp.terms)
        seeds.append((P.to_bytes(), search.default_generator(P).blob()))
    return seeds


def _record(prog: bytes, gen) -> bytes:
    out = struct.pack("<I", len(prog)) + prog
    if gen is None:
        return out + struct.pack("<I", 0xFFFFFFFF)
    g = np.asarray(gen, dtype=np.uint32)
    return out + struct.pack("<I", len(g)) + g.tobytes()


def _mutate_words(data, words: np.ndarray, label: str, body: int) -> np.ndarray:
    """Word-level mutation.  Half the mutants keep the length and header (in-place edits of
    the records after word ``body``), so they get past the framing checks and exercise the
    per-node / per-spec validation, the specialiser and the JIT emitter."""
    w = words.copy()
    if data.draw(st.booleans(), label=f"{label}.inplace") and len(w) > body:
        for _ in range(data.draw(st.integers(1, 3), label=f"{label}.n")):
            i = data.draw(st.integers(body, len(w) - 1), label=f"{label}.i")
            v = data.draw(st.one_of(st.sampled_from(BOUNDARY), st.integers(0, 0xFFFFFFFF),
                                    st.integers(0, 31).map(lambda b, x=int(w[i]): x ^ (1 << b))), label=f"{label}.v")
            w[i] = v
        return w
    for _ in range(data.draw(st.integers(1, 6), label=f"{label}.n")):
        kind = data.draw(st.integers(0, 6), label=f"{label}.kind")
        n = len(w)
        if kind <= 2 and n:
            # bias towards the header and the first records, where the counts live
            i = data.draw(st.one_of(st.integers(0, min(n, 24) - 1), st.integers(0, n - 1)), label=f"{label}.i")
            if kind == 0:
                w[i] ^= np.uint32(1 << data.draw(st.integers(0, 31)))
            elif kind == 1:
                w[i] = data.draw(st.sampled_from(BOUNDARY))
            else:
                w[i] = data.draw(st.integers(0, 0xFFFFFFFF))
        elif kind == 3 and n:
            w = w[:data.draw(st.integers(0, n - 1))]  # truncate
        elif kind == 4:
            extra = data.draw(st.lists(st.sampled_from(BOUNDARY), min_size=1, max_size=16))
            w = np.concatenate([w, np.array(extra, dtype=np.uint32)])
        elif kind == 5 and n > 2:
            a = data.draw(st.integers(0, n - 2))
            b = data.draw(st.integers(a + 1, min(n, a + 16)))
            at = data.draw(st.integers(0, n - 1))
            w = np.concatenate([w[:at], w[a:b], w[at:]])  # splice a copy of a run
        elif kind == 6 and n > 1:
            i, j = data.draw(st.integers(0, n - 1)), data.draw(st.integers(0, n - 1))
            w[i], w[j] = w[j], w[i]
    return w


def test_fuzz_parsers_under_asan_ubsan(fuzz_bin):
    seeds = _seeds()
    records = [_record(p, g) for p, g in seeds] + [_record(p, None) for p, _ in seeds]
    mutants = []

    @settings(max_examples=N_MUTANTS, deadline=None, database=None, derandomize=True,
              suppress_health_check=list(HealthCheck))
    @given(st.data())
    def collect(data):
        prog, gen = seeds[data.draw(st.integers(0, len(seeds) - 1), label="seed")]
        target = data.draw(st.integers(0, 3), label="target")  # 0 prog, 1 gen, 2 both, 3 prog without gen
        pw = np.frombuffer(prog, dtype=np.uint32)
        if target in (0, 2, 3):
            pw = _mutate_words(data, pw, "prog", 16)
        g = None if target == 3 else (_mutate_words(data, gen, "gen", 4) if target in (1, 2) else gen)
        tail = data.draw(st.sampled_from([0, 0, 0, 0, 1, 2, 3]), label="tail")  # byte-level truncation (non-word lengths)
        pb = pw.tobytes()
        mutants.append(_record(pb[:len(pb) - tail] if tail else pb, g))

    collect()
    assert len(mutants) >= min(N_MUTANTS, 1000)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:allocator_may_return_null=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([str(fuzz_bin)], input=b"".join(records + mutants), capture_output=True, env=env, timeout=900)
    err = r.stderr.decode(errors="replace")
    assert r.returncode == 0 and "Sanitizer" not in err and "runtime error" not in err, err[-4000:]
    counts = dict(kv.split("=") for kv in r.stdout.decode().split())
    print("fuzz:", counts)
    assert int(counts["records"]) == len(records) + len(mutants)
    # every seed lowers, and its generator parses and specialises
    assert int(counts["lowered"]) >= 2 * len(seeds) and int(counts["gen_ok"]) >= len(seeds)


def test_fuzz_seeds_alone_accepted(fuzz_bin):
    seeds = _seeds()
    r = subprocess.run([str(fuzz_bin)], input=b"".join(_record(p, g) for p, g in seeds), capture_output=True,
                       timeout=300, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=0"))
    assert r.returncode == 0, r.stderr.decode()[-3000:]
    counts = dict(kv.split("=") for kv in r.stdout.decode().split())
    assert counts == {"records": str(len(seeds)), "lowered": str(len(seeds)), "gen_ok": str(len(seeds)),
                      "specialised": str(2 * len(seeds))}
