"""Regenerate the committed golden fixtures from the reference's own test data.

Run HERE only (the GPU box has no /root/reference):

    python tests/golden/make_golden.py /root/reference

It copies DATA, never source: inputs and expected outputs that the reference's
tests hold.

* ``vmtests.json``  — ethereum/tests VMTests vectors the reference replays in
  ``tests/laser/evm_testsuite/evm_test.py:109-188`` (exec code/data/caller/value,
  pre storage, expected post storage; ``post == null`` when the test expects an
  exceptional halt).  The reference's ignore list (``evm_test.py:33-60``) is
  recorded per vector.
* ``eip145.json``   — the concrete SHL/SHR/SAR vectors parametrised in
  ``tests/instructions/{shl,shr,sar}_test.py`` (value, shift, expected).  They are
  read with ``ast.literal_eval`` of the parametrize tuples (no code is executed).
* ``keccak_kat.json`` — Keccak-256 known answers the reference pins:
  ``keccak("")`` (``keccak_function_manager.py:80`` and ``vmSha3Test/sha3_0.json``),
  the four-byte selectors of ``tests/cmd_line_test.py:27-29`` and
  ``tests/testdata/inputs/suicide.sol.o`` / ``README.md:54-75`` (message text is
  the Solidity signature; the selector is the expected first 4 bytes).
"""
import ast
import json
import sys
from pathlib import Path

HERE = Path(__file__).parent

VM_DIRS = [
    "vmArithmeticTest",
    "vmBitwiseLogicOperation",
    "vmSha3Test",
    "vmPushDupSwapTest",
    "vmIOandFlowOperations",
    "vmEnvironmentalInfo",
    "vmRandomTest",
    "vmTests",
    "vmSystemOperations",
]

# evm_test.py:33-60
IGNORED = {
    "gas0", "gas1", "log1MemExp",
    "BlockNumberDynamicJumpi0", "BlockNumberDynamicJumpi1", "BlockNumberDynamicJump0_jumpdest2",
    "DynamicJumpPathologicalTest0", "BlockNumberDynamicJumpifInsidePushWithJumpDest",
    "BlockNumberDynamicJumpiAfterStop", "BlockNumberDynamicJumpifInsidePushWithoutJumpDest",
    "BlockNumberDynamicJump0_jumpdest0", "BlockNumberDynamicJumpi1_jumpdest",
    "BlockNumberDynamicJumpiOutsideBoundary", "DynamicJumpJD_DependsOnJumps1",
    "loop_stacklimit_1020", "loop_stacklimit_1021",
    "jumpTo1InstructionafterJump", "sstore_load_2", "jumpi_at_the_end",
}


def vmtests(ref: Path):
    out = {}
    for d in VM_DIRS:
        for f in sorted((ref / "tests/laser/evm_testsuite/VMTests" / d).glob("*.json")):
            top = json.loads(f.read_text())
            for name, data in top.items():
                ex = data["exec"]
                addr = ex["address"]
                pre = data["pre"].get(addr, {})
                post = data.get("post")
                post_storage = None
                if post:
                    post_storage = post.get(addr, {}).get("storage", {})
                out[name] = {
                    "dir": d,
                    "code": ex["code"][2:],
                    "data": ex["data"][2:],
                    "caller": ex["caller"],
                    "origin": ex["origin"],
                    "address": addr,
                    "value": ex["value"],
                    "gasPrice": ex["gasPrice"],
                    "pre_storage": pre.get("storage", {}),
                    "post_storage": post_storage,
                    "reference_ignored": name in IGNORED,
                }
    return out


def _parametrize_tuples(path: Path, argnames: str):
    tree = ast.parse(path.read_text())
    for node in ast.walk(tree):
        if isinstance(node, ast.Call) and getattr(node.func, "attr", "") == "parametrize":
            if node.args and isinstance(node.args[0], ast.Constant) and node.args[0].value.replace(" ", "") == argnames:
                return ast.literal_eval(node.args[1])
    raise RuntimeError(f"no parametrize({argnames}) in {path}")


def eip145(ref: Path):
    out = {}
    for op in ("shl", "shr", "sar"):
        rows = _parametrize_tuples(ref / f"tests/instructions/{op}_test.py", "val1,val2,expected")
        out[op] = [{"value": r[0], "shift": r[1], "expected": r[2]} for r in rows]
    return out


def keccak_kat(vm):
    kats = [
        {"msg_hex": "", "digest": "0xc5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470",
         "source": "keccak_function_manager.py:80; vmSha3Test/sha3_0.json"},
    ]
    # selectors pinned by the reference's fixtures (first 4 bytes only)
    for sig, sel, src in [
        ("setOwner(address)", "0x13af4035", "tests/cmd_line_test.py:27-29"),
        ("kill(address)", "0xcbf0b0c0", "tests/testdata/inputs/suicide.sol.o"),
    ]:
        kats.append({"msg_hex": sig.encode().hex(), "selector": sel, "source": src})
    return kats


def main():
    ref = Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
    vm = vmtests(ref)
    (HERE / "vmtests.json").write_text(json.dumps(vm, indent=0, sort_keys=True))
    (HERE / "eip145.json").write_text(json.dumps(eip145(ref), indent=1))
    (HERE / "keccak_kat.json").write_text(json.dumps(keccak_kat(vm), indent=1))
    print(f"vmtests: {len(vm)} vectors")


if __name__ == "__main__":
    main()
