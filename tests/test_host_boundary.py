"""Host-side checks of the C-ABI boundary and the flattener — CPU only (no compute
call needs a GPU here)."""
import ctypes
import re
from pathlib import Path

import pytest

from mythril_amd import native, ssa
from mythril_amd.smt import (Array, BVAddNoOverflow, BVMulNoOverflow, BVSubNoUnderflow, Concat, Function, If, K,
                             Not, UDiv, UGE, UGT, ULT, symbol_factory)
from mythril_amd.smt import terms as T

ROOT = Path(__file__).resolve().parent.parent
HEADER = (ROOT / "include" / "mythgpu.h").read_text()


@pytest.fixture(scope="module")
def lib():
    from mythril_amd import build

    build.build()
    return native.load_library()


def test_header_opcodes_match_flattener():
    enum = dict(re.findall(r"MG_OP_([A-Z_]+) = (\d+)", HEADER))
    enum.pop("COUNT")
    assert {k: int(v) for k, v in enum.items()} == ssa.OPS


def test_library_exports_every_declared_symbol(lib):
    declared = set(re.findall(r"^\s*(?:int|void|const char\*)\s+(mg_\w+)\(", HEADER, re.M))
    assert declared == set(native.EXPORTS)
    for name in declared:
        assert hasattr(lib, name), name
    assert lib.mg_version() == 2


def test_init_without_device_fails_loudly(lib):
    if Path("/dev/kfd").exists():
        pytest.skip("a GPU is present")
    with pytest.raises(native.EngineError):
        native.Engine(0)


def _bec_constraints():
    """BECToken batchOverflow shape."""
    cnt = symbol_factory.BitVecSym("cnt", 256)
    value = symbol_factory.BitVecSym("value", 256)
    sender = symbol_factory.BitVecSym("sender_1", 256)
    storage = Array("Storage", 256, 256)
    keccak = Function("keccak256_512", 512, 256)
    slot = keccak(Concat(sender, symbol_factory.BitVecVal(0, 256)))
    amount = cnt * value
    return [
        Not(BVMulNoOverflow(cnt, value, False)),
        UGT(cnt, symbol_factory.BitVecVal(0, 256)),
        ULT(cnt, symbol_factory.BitVecVal(21, 256)),
        UGT(value, symbol_factory.BitVecVal(0, 256)),
        UGE(storage[slot], amount),
    ]


def test_program_check_and_cost(lib):
    cs = _bec_constraints()
    P = ssa.flatten([c.raw for c in cs])
    info = native.check_program(P.to_bytes())
    assert info.n_roots == 5
    assert info.n_coords == len(P.coords) == 5  # cnt, value, sender, keccak site, storage site
    assert info.coord_words == 8 * 4 + 8
    # MUL 128 + UMUL_NOOVF 256 + 4 compares ... : cost table is deterministic
    assert info.limb_ops > 128 + 256
    assert info.value_words < 160


def test_unsupported_wide_arithmetic(lib):
    x = T.BitVecVar("x", 512)
    t = T.eq(T.bvbin("bvmul", x, x), x)
    P = ssa.flatten([t])
    with pytest.raises(native.EngineUnsupported):
        native.check_program(P.to_bytes())


def test_malformed_program_rejected(lib):
    x = symbol_factory.BitVecSym("x", 256)
    blob = bytearray(ssa.flatten([(x == 1).raw]).to_bytes())
    blob[0] ^= 0xFF
    with pytest.raises(native.EngineError):
        native.check_program(bytes(blob))
    with pytest.raises(native.EngineError):
        native.check_program(bytes(ssa.flatten([(x == 1).raw]).to_bytes())[:-4])


def test_flatten_sites_and_lazy_inverse():
    x = symbol_factory.BitVecSym("x", 256)
    f = Function("keccak256_256", 256, 256)
    inv = Function("keccak256_256-1", 256, 256)
    c = inv(f(x)) == x
    P = ssa.flatten([c.raw])
    kinds = [co.kind for co in P.coords]
    assert kinds == [ssa.COORD_SCALAR, ssa.COORD_UF_SITE, ssa.COORD_UF_SITE]
    inv_node = P.coords[2].node
    assert P.nodes[inv_node][7] == P.coords[0].node  # lazy default = x


def test_flatten_select_over_store_chain():
    s = K(256, 256, 0)
    a = symbol_factory.BitVecSym("a", 256)
    s[a] = symbol_factory.BitVecVal(5, 256)
    c = s[symbol_factory.BitVecVal(3, 256)] == 5
    P = ssa.flatten([c.raw])
    assert all(co.kind == ssa.COORD_SCALAR for co in P.coords)  # K() base: no site


def test_addnooverflow_expands_like_z3():
    a = symbol_factory.BitVecSym("a", 256)
    b = symbol_factory.BitVecSym("b", 256)
    t = BVAddNoOverflow(a, b, False).raw
    assert t.op == "eq" and t.args[0].op == "extract" and t.args[0].params == (256, 256)
    assert BVSubNoUnderflow(a, b, False).raw.op == "bvule"


def test_prefix_incremental_flatten_is_byte_identical():
    """FlattenCache extends the longest cached root prefix;
    the program must equal a fresh flatten of the whole tuple, byte for byte."""
    import random

    from mythril_amd import workloads

    fc = ssa.FlattenCache(capacity=64)
    rng = random.Random(3)
    for name, fn in workloads.WORKLOADS.items():
        roots = [c.raw for c in fn()]
        for _ in range(4):  # a random walk of prefixes, as sibling states produce
            k = rng.randint(1, len(roots))
            assert fc.flatten(roots[:k]).to_bytes() == ssa.flatten(roots[:k]).to_bytes(), name
        P = fc.flatten(roots)
        assert P.to_bytes() == ssa.flatten(roots).to_bytes(), name
        P.set_watch([0])  # callers may mutate what they get; the cache must not see it
        assert fc.flatten(roots).watch == []
    assert fc.hits > 0


def test_flatten_cache_survives_unsupported_extension():
    """A query that fails to flatten (ssa.Unsupported) must leave the cached
    prefix untouched: the next extension of that prefix is still byte-identical."""
    from mythril_amd import workloads

    roots = [c.raw for c in workloads.WORKLOADS["bectoken_batch_overflow"]()]
    fc = ssa.FlattenCache()
    fc.flatten(roots[:-1])
    wide = T.BitVecVar("too_wide", ssa.MG_MAX_WIDTH + 8)
    bad = T.eq(wide, T.BitVecVal(1, ssa.MG_MAX_WIDTH + 8))
    with pytest.raises(ssa.Unsupported):
        fc.flatten(roots[:-1] + [bad])
    assert fc.flatten(roots).to_bytes() == ssa.flatten(roots).to_bytes()


def test_same_name_two_sorts_is_unsupported():
    """BitVec('x', 8) and BitVec('x', 256) are different z3 constants, but Model.scalars is
    keyed by name: the flattener must refuse the query (the caller falls back to z3)
    rather than return a model where one value overwrote the other."""
    x8 = T.BitVecVar("x", 8)
    x256 = T.BitVecVar("x", 256)
    roots = [T.eq(x8, T.BitVecVal(3, 8)), T.eq(x256, T.BitVecVal(1 << 200, 256))]
    with pytest.raises(ssa.Unsupported, match="two sorts"):
        ssa.flatten(roots)
    # incremental: the second sort arrives in an extension of a cached prefix
    fc = ssa.FlattenCache()
    fc.flatten(roots[:1])
    with pytest.raises(ssa.Unsupported, match="two sorts"):
        fc.flatten(roots)
    # arrays / UFs: same name at two sorts
    a = T.ArrayVar("m", 256, 256)
    b = T.ArrayVar("m", 256, 8)
    with pytest.raises(ssa.Unsupported, match="two sorts"):
        ssa.flatten([T.eq(T.select(a, x256), T.BitVecVal(1, 256)), T.eq(T.select(b, x256), T.BitVecVal(1, 8))])
    f1 = Function("f", 256, 256)
    f2 = Function("f", 256, 8)
    y = symbol_factory.BitVecSym("y", 256)
    with pytest.raises(ssa.Unsupported, match="two sorts"):
        ssa.flatten([(f1(y) == 1).raw, (f2(y) == 1).raw])
    # one name at one sort used many times is fine
    assert len(ssa.flatten([roots[1], T.eq(x256, x256)]).scalar_coords()) == 1


@pytest.mark.parametrize("start,count,n", [(0, 1 << 20, 4), (13, 100_000, 3), (64, 64, 8), (5, 3, 4), (0, 0, 2),
                                           (1 << 40, (1 << 26) + 7, 8), (63, 2, 2), (100, 1, 1)])
def test_split_range_chunk_to_device(lib, start, count, n):
    """mg_split_range (the multi-device mg_search / mg_jit_search split): contiguous slices
    in device order that tile [start, start+count) exactly, boundaries on aligned 64-index
    groups (one wave's group key: a group is never shared by two devices), balanced to
    within one group."""
    sl = native.split_range(start, count, n)
    assert len(sl) == n
    pos = start
    sizes = []
    for s0, c in sl:
        if c == 0:
            continue
        assert s0 == pos  # contiguous, in order
        if s0 != start:
            assert s0 % 64 == 0
        pos = s0 + c
        groups = ((s0 + c - 1) >> 6) - (s0 >> 6) + 1
        sizes.append(groups)
    assert pos == start + count
    if sizes:
        assert max(sizes) - min(sizes) <= 2
    with pytest.raises(native.EngineError):
        native.split_range(0, 10, 0)


def test_bench_gpus_without_launcher_needs_the_devices():
    """``bench.py --gpus N`` with no torch.distributed launcher opens N devices in one process
    (the product's in-shim split); with fewer GPUs visible it exits 2 before touching a GPU."""
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    env = {k: v for k, v in __import__("os").environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 2, r.stderr[-2000:]
    assert "--gpus 2 but only 0 GPU(s) visible" in r.stderr
    assert r.stdout == ""


def test_model_from_assignment_matches_model_from_sites():
    """The model read back from mg_search's assign_out rows (literal site keys and AUX-sliced
    calldata bytes filled in on the host, ``search._model_layout``) equals the generic
    ``ssa.model_from_sites`` of the full per-site key / base values, duplicate keys included
    (random coordinate and key values; the watch rows are what the kernel writes for them)."""
    import random

    import numpy as np

    from mythril_amd import search, workloads

    rng = random.Random(5)
    for name, fn in workloads.WORKLOADS.items():
        roots = [c.raw for c in fn()]
        P, _ = search.prepare(roots)
        assert search.prepare(roots)[0] is P  # the prepared query is cached whole
        entries, widths = search.model_watch(P)
        n_sites_lit = sum(1 for c in P.sites if search._const_node_value(P, P.site_key_node[c.index]) is not None)
        assert len(entries) == len(P.scalar_coords()) + len({a for a, _ in P.aux_slice.values()}) + \
            2 * len(P.sites) - n_sites_lit - len(P.aux_slice), name
        node_of = {c.node: c for c in P.coords if c.kind in (ssa.COORD_SCALAR, ssa.COORD_AUX)}
        for trial in range(3):
            draw = (lambda w: rng.randrange(3)) if trial == 2 else rng.getrandbits  # trial 2: colliding keys
            vals_c = {c.index: draw(c.width) for c in P.coords}
            # a key node's value (what the kernel computes for it): literal, or any value
            key_val = {}
            for c in P.sites:
                k = P.site_key_node[c.index]
                lit = search._const_node_value(P, k)
                if k in node_of:
                    key_val[k] = vals_c[node_of[k].index]
                elif k not in key_val:
                    key_val[k] = lit if lit is not None else draw(P.node_width[k])
            keys = {c.index: key_val[P.site_key_node[c.index]] for c in P.sites}
            bases = {}
            for c in P.sites:
                sl = P.aux_slice.get(c.index)
                bases[c.index] = (vals_c[sl[0]] >> sl[1]) & 0xFF if sl else vals_c[c.index]
            want = ssa.model_from_sites(P, {c.index: vals_c[c.index] for c in P.scalar_coords()}, keys, bases)
            # the watch rows the kernel writes: one value per entry
            row_vals = []
            for e in entries:
                if e & 0x80000000:
                    row_vals.append(bases[e & 0x7FFFFFFF])
                elif e in node_of:
                    row_vals.append(vals_c[node_of[e].index])
                else:
                    row_vals.append(key_val[e])
            assign = []
            for v, w in zip(row_vals, widths):
                assign += [(v >> (32 * j)) & 0xFFFFFFFF for j in range(ssa.limbs(w))]
            got = search.model_from_assignment(P, np.array(assign or [0], dtype=np.uint32))
            assert got == want, name
