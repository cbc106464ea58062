"""Pin the oracle (CPU restatement of z3 model.eval + LASER opcode semantics)
against the reference's own golden vectors — CPU only.

* Keccak-256 KATs: keccak_function_manager.py:80, vmSha3Test, selectors in
  tests/cmd_line_test.py:27-29 and tests/testdata/inputs/suicide.sol.o.
* EIP-145 SHL/SHR/SAR vectors: tests/instructions/{shl,shr,sar}_test.py.
* VMTests post-state storage through LASER's opcode->term mapping
  (tests/laser/evm_testsuite/evm_test.py:109-188).
"""
import pytest

from helpers import load_json, vmtest_cases
from mythril_amd.smt import LShR, symbol_factory
from oracle.bv import OracleModel, evaluate
from oracle.keccak import keccak256, keccak256_int

BVV = symbol_factory.BitVecVal


def test_keccak_kats():
    for kat in load_json("keccak_kat.json"):
        d = keccak256(bytes.fromhex(kat["msg_hex"]))
        if "digest" in kat:
            assert "0x" + d.hex() == kat["digest"]
        else:
            assert "0x" + d[:4].hex() == kat["selector"]


def test_keccak_empty_matches_reference_constant():
    # keccak_function_manager.py:75-81 stores keccak256("") in decimal
    assert keccak256_int(b"") == 89477152217924674838424037953991966239322087453347756267410168184682657981552


@pytest.mark.parametrize("op", ["shl", "shr", "sar"])
def test_eip145_vectors(op):
    rows = load_json("eip145.json")[op]
    assert rows
    for r in rows:
        value, shift = BVV(int(r["value"], 16), 256), BVV(int(r["shift"], 16), 256)
        term = {"shl": value << shift, "shr": LShR(value, shift), "sar": value >> shift}[op]
        assert evaluate(term.raw, OracleModel()) == int(r["expected"], 16), r


def test_vmtests_post_storage():
    """Every VMTests vector with a post-state (429: the reference's non-ignored set) replays to its
    expected storage words; input-dependent jumps followed along the concrete path leave path
    constraints that hold for the vector's inputs."""
    cases = vmtest_cases()
    assert len(cases) == 429
    dirs = {}
    for name, v, r in cases:
        from mythril_amd.replay import replay_assignment

        scal, arrs = replay_assignment(v)
        m = OracleModel(scal, arrs)
        for k, x in v["post_storage"].items():
            assert evaluate(r.storage_word(int(k, 16)).raw, m) == int(x, 16), (name, k)
        for c in r.path:
            assert evaluate(c, m) == 1, name
        dirs[v["dir"]] = dirs.get(v["dir"], 0) + 1
    # every arithmetic / bitwise / sha3 vector with a post-state is covered
    assert dirs["vmArithmeticTest"] >= 190
    assert dirs["vmBitwiseLogicOperation"] >= 59
    assert dirs["vmSha3Test"] >= 12


def test_smt_division_semantics():
    """SMT-LIB total division, as z3 evaluates LASER's UDiv/URem/SDiv/SRem/SMod terms."""
    from mythril_amd.smt import SRem, UDiv, URem

    x = symbol_factory.BitVecSym("x", 256)
    zero = BVV(0, 256)
    M = (1 << 256) - 1
    m = OracleModel({"x": 7})
    assert evaluate(UDiv(x, zero).raw, m) == M
    assert evaluate(URem(x, zero).raw, m) == 7
    assert evaluate((x / zero).raw, m) == M
    assert evaluate((x / zero).raw, OracleModel({"x": M})) == 1  # negative dividend -> 1
    assert evaluate(SRem(x, zero).raw, m) == 7
    assert evaluate((x % zero).raw, m) == 7
    mn = 1 << 255
    assert evaluate((x / BVV(M, 256)).raw, OracleModel({"x": mn})) == mn  # -2^255 / -1 wraps


def test_jumpi_path_constraint_is_lasers():
    """An input-dependent JUMPI followed along the concrete path records LASER's branch constraint —
    ``cond != 0`` taken, ``cond == 0`` not taken (``instructions.py:1565-1571``) — and the target is a
    decision only when the branch is taken.  Code: CALLDATALOAD(0) as the condition, JUMPI to 7."""
    from mythril_amd.replay import replay
    from mythril_amd.smt import terms as T

    code = "600035600757005b00"  # PUSH1 0 CALLDATALOAD PUSH1 7 JUMPI STOP JUMPDEST STOP
    for word, taken in ((5, True), (0, False)):
        data = word.to_bytes(32, "big")
        arrs = {"calldata": ({i: b for i, b in enumerate(data)}, 0)}
        m = OracleModel({"calldatasize": 32}, arrs)
        r = replay(code, data, follow=lambda t, m=m: evaluate(t, m))
        assert len(r.path) == 1, r.path
        c = r.path[0]
        assert (c.op == "not") == taken, c.op  # Not(cond == 0) taken, cond == 0 not taken
        assert evaluate(c, m) == 1
        other = OracleModel({"calldatasize": 32}, {"calldata": ({31: 0 if taken else 9}, 0)})
        assert evaluate(c, other) == 0  # the constraint is the branch, not the concrete value


def test_jumpi_symbolic_target_is_skipped_as_laser_does():
    """A JUMPI whose target is input-dependent is skipped with no branch constraint, as LASER's
    ``jumpi_`` does when ``get_concrete_int`` raises (``instructions.py:1549-1555``): execution
    falls through whatever the condition.  Code: CALLDATALOAD(0) as the target, condition 1, then
    SSTORE(0, 1) on the fall-through path, and a JUMPDEST at 12 that the target would reach."""
    from mythril_amd.replay import replay

    # PUSH1 1 PUSH1 0 CALLDATALOAD JUMPI PUSH1 1 PUSH1 0 SSTORE STOP JUMPDEST STOP
    code = "6001600035576001600055005b00"
    for word in (12, 0, 7):
        data = word.to_bytes(32, "big")
        arrs = {"calldata": ({i: b for i, b in enumerate(data)}, 0)}
        m = OracleModel({"calldatasize": 32}, arrs)
        r = replay(code, data, follow=lambda t, m=m: evaluate(t, m))
        assert r.path == [], r.path
        assert evaluate(r.storage_word(0).raw, m) == 1  # fell through to the SSTORE
