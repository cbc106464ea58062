"""Concrete transaction replay -> constraint program (LASER opcode semantics).

A *replay request* is one message call with concrete inputs (code, calldata,
caller, value, pre-state storage).  The reference executes it with
``transaction/concolic.py:15-62`` and checks post-state storage in
``tests/laser/evm_testsuite/evm_test.py:109-188``.  Here the call is executed
*once, symbolically over its inputs* along its single concrete path, building
terms with exactly LASER's opcode -> term mapping (``instructions.py``, cited per
opcode below); the resulting program (post-storage words as functions of the
input coordinates) is then evaluated on the GPU for the concrete inputs — and,
for free, for any batch of other inputs.

Inputs become coordinates: ``caller``, ``origin``, ``address``, ``callvalue``,
``gasprice``, ``calldatasize`` (256-bit scalars) and the array ``calldata``
(BitVec(256) -> BitVec(8)).  Control decisions (jump targets, memory offsets,
SHA3 lengths, the DIV/MOD "divisor == 0" checks) are taken on the host by
literal folding, exactly where LASER takes them with ``z3.simplify``; a decision
that depends on an input raises :class:`ReplayUnsupported`.

An input-dependent jump (a JUMP target or JUMPI condition computed from calldata) is followed
along the concrete path when the caller passes ``follow`` (term -> its value under the request's
concrete inputs, e.g. :func:`engine_follow`, which evaluates it on the GPU): the replay then takes
that branch and records the decision as a path constraint (``ReplayResult.path``), so the program is
exactly LASER's path condition plus the post-state of that path — as concolic execution takes the
concrete branch (``transaction/concolic.py:15-62``).  Without ``follow`` such a request is refused.

Two documented departures, both for concrete execution only: SHA3 of memory
becomes the engine's real ``keccak256`` term (LASER hashes concrete data on the
host, ``keccak_function_manager.py:44-57``), and EXP becomes ``bvexp`` (LASER
computes ``pow`` on the host for concrete operands, ``instructions.py:622-629``).
"""
from __future__ import annotations

from typing import Dict, List, Optional

from . import smt as S
from .smt import terms as T
from .smt import BitVec, Bool, If, symbol_factory

TT256 = 1 << 256
TT256M1 = TT256 - 1
BVV = symbol_factory.BitVecVal


class ReplayUnsupported(Exception):
    """The request needs an input-dependent control decision or an opcode
    outside the replay subset."""


class ExceptionalHalt(Exception):
    """EVM exceptional halt (stack underflow, invalid opcode, bad jump)."""


def disassemble(code: bytes):
    """(pc, opcode byte, push immediate or None) list."""
    out, pc = [], 0
    while pc < len(code):
        op = code[pc]
        if 0x60 <= op <= 0x7F:
            n = op - 0x5F
            imm = int.from_bytes(code[pc + 1: pc + 1 + n].ljust(n, b"\0"), "big")
            out.append((pc, op, imm))
            pc += 1 + n
        else:
            out.append((pc, op, None))
            pc += 1
    return out


class ReplayResult:
    def __init__(self, storage: S.BaseArray, halted: str, inputs: Dict[str, T.Term], touched, path=()):
        self.storage = storage
        self.halted = halted
        self.inputs = inputs
        self.touched = touched  # storage keys written (concrete ints where foldable)
        self.path = list(path)  # Bool terms: the input-dependent decisions taken (``follow``)

    def storage_word(self, key: int) -> BitVec:
        """Post-state storage word at a concrete key (``account.storage[key]``)."""
        return self.storage[BVV(key, 256)]


def _pop_bitvec(stack) -> BitVec:
    """``util.pop_bitvec`` (util.py:67-88) without the simplify: Bool -> If(b,1,0)."""
    if not stack:
        raise ExceptionalHalt("stack underflow")
    item = stack.pop()
    if isinstance(item, Bool):
        return If(item, BVV(1, 256), BVV(0, 256))
    if isinstance(item, int):
        return BVV(item, 256)
    return item


def _pop(stack):
    if not stack:
        raise ExceptionalHalt("stack underflow")
    return stack.pop()


def _concrete(x, what: str) -> int:
    """``util.get_concrete_int`` (util.py:91-109) via literal folding."""
    if isinstance(x, int):
        return x
    if isinstance(x, Bool):
        v = x.value
    else:
        v = x.value
    if v is None:
        raise ReplayUnsupported(f"input-dependent {what}")
    return int(v)


def _as_bv(x) -> BitVec:
    if isinstance(x, Bool):
        return If(x, BVV(1, 256), BVV(0, 256))
    if isinstance(x, int):
        return BVV(x, 256)
    return x


class _Memory:
    """Byte-addressed memory of 8-bit terms (``state/memory.py:56-115``)."""

    def __init__(self):
        self.bytes: Dict[int, BitVec] = {}
        self.size = 0

    def extend(self, off: int, n: int):
        if n and off + n > self.size:
            self.size = ((off + n + 31) // 32) * 32

    def byte(self, i: int) -> BitVec:
        return self.bytes.get(i, BVV(0, 8))

    def word(self, off: int) -> BitVec:
        return S.Concat([self.byte(off + i) for i in range(32)])

    def write_word(self, off: int, value):
        value = _as_bv(value)
        for i in range(32):
            hi = 255 - 8 * i
            self.bytes[off + i] = S.Extract(hi, hi - 7, value)


def replay(code_hex: str, calldata: bytes = b"", pre_storage: Optional[Dict[int, int]] = None,
           max_steps: int = 10000, follow=None) -> ReplayResult:
    code = bytes.fromhex(code_hex)
    ins = disassemble(code)
    pc_index = {pc: k for k, (pc, _, _) in enumerate(ins)}
    jumpdests = {pc for pc, op, _ in ins if op == 0x5B}

    inputs = {n: T.BitVecVar(n, 256) for n in ("caller", "origin", "address", "callvalue", "gasprice", "calldatasize")}
    calldata_arr = S.Array("calldata", 256, 8)
    size = BitVec(inputs["calldatasize"])

    storage = S.K(256, 256, 0)  # concrete_storage=True accounts (account.py:26-29)
    for k, v in (pre_storage or {}).items():
        storage[BVV(k, 256)] = BVV(v, 256)

    stack: List = []
    mem = _Memory()
    touched = []
    path: List[T.Term] = []

    def decide(x, what: str) -> int:
        """A control decision: folded where LASER's simplify folds it, else followed along the
        concrete path (``follow``) with the decision kept as a path constraint."""
        x = _as_bv(x)
        if x.value is not None:
            return int(x.value)
        if follow is None:
            raise ReplayUnsupported(f"input-dependent {what}")
        v = int(follow(x.raw)) & TT256M1
        path.append(T.eq(x.raw, BVV(v, 256).raw))
        return v

    def branch(cond) -> bool:
        """A JUMPI condition: folded, or followed with LASER's branch constraint kept — ``cond != 0``
        on the taken branch, ``cond == 0`` on the fall-through (``instructions.py:1565-1571``)."""
        cond = _as_bv(cond)
        if cond.value is not None:
            return int(cond.value) != 0
        if follow is None:
            raise ReplayUnsupported("input-dependent JUMPI condition")
        taken = (int(follow(cond.raw)) & TT256M1) != 0
        zero = BVV(0, 256).raw
        path.append(T.not_(T.eq(cond.raw, zero)) if taken else T.eq(cond.raw, zero))
        return taken

    def result(halted: str) -> ReplayResult:
        return ReplayResult(storage, halted, inputs, touched, path)
    k = 0
    steps = 0

    def cd_byte(item: BitVec) -> BitVec:
        # SymbolicCalldata._load (calldata.py:226-231): If(item < size, calldata[item], 0) — signed '<'
        return If(item < size, calldata_arr[item], BVV(0, 8))

    while True:
        steps += 1
        if steps > max_steps:
            raise ReplayUnsupported("step limit")
        if k >= len(ins):
            return result("stop")
        pc, op, imm = ins[k]
        k += 1
        if 0x60 <= op <= 0x7F:                       # PUSHn
            stack.append(BVV(imm, 256))
        elif 0x80 <= op <= 0x8F:                     # DUPn
            n = op - 0x7F
            if len(stack) < n:
                raise ExceptionalHalt("stack underflow")
            stack.append(stack[-n])
        elif 0x90 <= op <= 0x9F:                     # SWAPn
            n = op - 0x8F
            if len(stack) < n + 1:
                raise ExceptionalHalt("stack underflow")
            stack[-1], stack[-n - 1] = stack[-n - 1], stack[-1]
        elif op == 0x00:                             # STOP
            return result("stop")
        elif op == 0x01:                             # ADD  instructions.py:433-441
            stack.append(_pop_bitvec(stack) + _pop_bitvec(stack))
        elif op == 0x02:                             # MUL  :464-477
            stack.append(_pop_bitvec(stack) * _pop_bitvec(stack))
        elif op == 0x03:                             # SUB  :448-461
            stack.append(_pop_bitvec(stack) - _pop_bitvec(stack))
        elif op == 0x04:                             # DIV  :480-494 (concrete 0 divisor -> 0)
            a, b = _pop_bitvec(stack), _pop_bitvec(stack)
            stack.append(BVV(0, 256) if (b == 0) else S.UDiv(a, b))
        elif op == 0x05:                             # SDIV :497-511
            a, b = _pop_bitvec(stack), _pop_bitvec(stack)
            stack.append(BVV(0, 256) if (b == 0) else a / b)
        elif op == 0x06:                             # MOD  :514-525
            a, b = _pop_bitvec(stack), _pop_bitvec(stack)
            stack.append(BVV(0, 256) if (b == 0) else S.URem(a, b))
        elif op == 0x07:                             # SMOD :555-566 (SRem, sign of dividend)
            a, b = _pop_bitvec(stack), _pop_bitvec(stack)
            stack.append(BVV(0, 256) if (b == 0) else S.SRem(a, b))
        elif op == 0x08:                             # ADDMOD :569-581 (wraps at 2^256)
            a, b, m = _pop_bitvec(stack), _pop_bitvec(stack), _pop_bitvec(stack)
            stack.append(S.URem(S.URem(a, m) + S.URem(b, m), m))
        elif op == 0x09:                             # MULMOD :584-596 (wraps at 2^256)
            a, b, m = _pop_bitvec(stack), _pop_bitvec(stack), _pop_bitvec(stack)
            stack.append(S.URem(S.URem(a, m) * S.URem(b, m), m))
        elif op == 0x0A:                             # EXP  :599-631 -> bvexp (concrete replay)
            base, exp = _pop_bitvec(stack), _pop_bitvec(stack)
            stack.append(BitVec(T.bvexp(base.raw, exp.raw), base.annotations | exp.annotations))
        elif op == 0x0B:                             # SIGNEXTEND :634-662
            s0, s1 = _pop(stack), _as_bv(_pop(stack))
            s0 = _concrete(_as_bv(s0), "SIGNEXTEND byte index")
            if s0 <= 31:
                testbit = s0 * 8 + 7
                if not S.is_true(S.simplify((s1 & (1 << testbit)) == 0)):
                    stack.append(s1 | (TT256 - (1 << testbit)))
                else:
                    stack.append(s1 & ((1 << testbit) - 1))
            else:
                stack.append(s1)
        elif op == 0x10:                             # LT  :666-675
            stack.append(S.ULT(_pop_bitvec(stack), _pop_bitvec(stack)))
        elif op == 0x11:                             # GT  :678-688
            a, b = _pop_bitvec(stack), _pop_bitvec(stack)
            stack.append(S.UGT(a, b))
        elif op == 0x12:                             # SLT :691-700
            stack.append(_pop_bitvec(stack) < _pop_bitvec(stack))
        elif op == 0x13:                             # SGT :703-713
            stack.append(_pop_bitvec(stack) > _pop_bitvec(stack))
        elif op == 0x14:                             # EQ  :716-740
            a, b = _as_bv(_pop(stack)), _as_bv(_pop(stack))
            stack.append(a == b)
        elif op == 0x15:                             # ISZERO :743-758
            v = _pop(stack)
            e = S.Not(v) if isinstance(v, Bool) else (_as_bv(v) == 0)
            stack.append(If(e, BVV(1, 256), BVV(0, 256)))
        elif op == 0x16:                             # AND :330-351
            a, b = _as_bv(_pop(stack)), _as_bv(_pop(stack))
            stack.append(a & b)
        elif op == 0x17:                             # OR  :354-375
            a, b = _as_bv(_pop(stack)), _as_bv(_pop(stack))
            stack.append(a | b)
        elif op == 0x18:                             # XOR :378-387
            a, b = _as_bv(_pop(stack)), _as_bv(_pop(stack))
            stack.append(a ^ b)
        elif op == 0x19:                             # NOT :390-398  (TT256M1 - x)
            stack.append(BVV(TT256M1, 256) - _as_bv(_pop(stack)))
        elif op == 0x1A:                             # BYTE :401-430
            op0, op1 = _pop(stack), _as_bv(_pop(stack))
            index = _concrete(_as_bv(op0), "BYTE index")
            offset = (31 - index) * 8
            if offset >= 0:
                stack.append(S.Concat(BVV(0, 248), S.Extract(offset + 7, offset, op1)))
            else:
                stack.append(BVV(0, 256))
        elif op == 0x1B:                             # SHL :528-534
            shift, value = _pop_bitvec(stack), _pop_bitvec(stack)
            stack.append(value << shift)
        elif op == 0x1C:                             # SHR :537-543
            shift, value = _pop_bitvec(stack), _pop_bitvec(stack)
            stack.append(S.LShR(value, shift))
        elif op == 0x1D:                             # SAR :546-552
            shift, value = _pop_bitvec(stack), _pop_bitvec(stack)
            stack.append(value >> shift)
        elif op == 0x20:                             # SHA3 :1009-1048 -> keccak256 term
            off = _concrete(_as_bv(_pop(stack)), "SHA3 offset")
            ln = _concrete(_as_bv(_pop(stack)), "SHA3 length")
            if ln > 4096:
                raise ReplayUnsupported("SHA3 length")
            mem.extend(off, ln)
            if ln == 0:
                stack.append(BitVec(T.keccak256_empty()))
            else:
                data = mem.byte(off) if ln == 1 else S.Concat([mem.byte(off + i) for i in range(ln)])
                stack.append(BitVec(T.keccak256(data.raw)))
        elif op == 0x30:                             # ADDRESS
            stack.append(BitVec(inputs["address"]))
        elif op == 0x32:                             # ORIGIN
            stack.append(BitVec(inputs["origin"]))
        elif op == 0x33:                             # CALLER
            stack.append(BitVec(inputs["caller"]))
        elif op == 0x34:                             # CALLVALUE :762-773
            stack.append(BitVec(inputs["callvalue"]))
        elif op == 0x35:                             # CALLDATALOAD :775-789 (calldata.py:47-54)
            start = _as_bv(_pop(stack))
            stack.append(S.Concat([cd_byte(start + i) for i in range(32)]))
        elif op == 0x36:                             # CALLDATASIZE :791-807
            stack.append(size)
        elif op == 0x37:                             # CALLDATACOPY :881-893, _calldata_copy_helper :810-878
            mstart = _concrete(_as_bv(_pop(stack)), "CALLDATACOPY memory offset")
            dstart = _as_bv(_pop(stack))
            n = _concrete(_as_bv(_pop(stack)), "CALLDATACOPY size")
            if n > 4096 or mstart > 1 << 20:
                raise ReplayUnsupported("CALLDATACOPY size")
            if n > 0:
                mem.extend(mstart, n)
                for i in range(n):
                    mem.bytes[mstart + i] = cd_byte(dstart + i)
        elif op == 0x38:                             # CODESIZE
            stack.append(BVV(len(code), 256))
        elif op == 0x39:                             # CODECOPY :1061-1165, _code_copy_helper :1167-1227
            moff = _concrete(_as_bv(_pop(stack)), "CODECOPY memory offset")
            coff = _concrete(_as_bv(_pop(stack)), "CODECOPY code offset")
            n = _concrete(_as_bv(_pop(stack)), "CODECOPY size")
            if n > 4096 or moff > 1 << 20:
                raise ReplayUnsupported("CODECOPY size")
            mem.extend(moff, n)
            for i in range(n):
                if coff + i >= len(code):  # the reference stops at the end of the code (memory kept)
                    break
                mem.bytes[moff + i] = BVV(code[coff + i], 8)
        elif op == 0x3A:                             # GASPRICE
            stack.append(BitVec(inputs["gasprice"]))
        elif op == 0x50:                             # POP
            _pop(stack)
        elif op == 0x51:                             # MLOAD :1421-1435
            off = _concrete(_as_bv(_pop(stack)), "MLOAD offset")
            if off > 1 << 20:
                raise ReplayUnsupported("MLOAD offset")
            mem.extend(off, 32)
            stack.append(mem.word(off))
        elif op == 0x52:                             # MSTORE :1437-1453
            off = _concrete(_as_bv(_pop(stack)), "MSTORE offset")
            if off > 1 << 20:
                raise ReplayUnsupported("MSTORE offset")
            val = _pop(stack)
            mem.extend(off, 32)
            mem.write_word(off, val)
        elif op == 0x53:                             # MSTORE8 :1455-1476
            off = _concrete(_as_bv(_pop(stack)), "MSTORE8 offset")
            if off > 1 << 20:
                raise ReplayUnsupported("MSTORE8 offset")
            val = _as_bv(_pop(stack))
            mem.extend(off, 1)
            mem.bytes[off] = S.Extract(7, 0, val)
        elif op == 0x54:                             # SLOAD :1478-1489
            idx = _as_bv(_pop(stack))
            stack.append(storage[idx])
        elif op == 0x55:                             # SSTORE :1491-1501
            idx, val = _as_bv(_pop(stack)), _pop(stack)
            storage[idx] = _as_bv(val)
            touched.append(idx)
        elif op == 0x56:                             # JUMP
            dest = decide(_pop(stack), "JUMP target")
            if dest not in jumpdests:
                raise ExceptionalHalt("bad jump")
            k = pc_index[dest]
        elif op == 0x57:                             # JUMPI (:1537-1585)
            target = _as_bv(_pop(stack))
            cond = _pop(stack)
            # LASER reads the target with get_concrete_int first: a symbolic one raises TypeError and
            # the JUMPI is skipped — pc + 1, no branch constraint, the condition never looked at
            # ("Skipping JUMPI to invalid destination.", :1549-1555)
            if target.value is not None:
                c = branch(cond)
                if c:
                    dest = int(target.value)
                    if dest not in jumpdests:
                        raise ExceptionalHalt("bad jump")
                    k = pc_index[dest]
        elif op == 0x58:                             # PC
            stack.append(BVV(pc, 256))
        elif op == 0x59:                             # MSIZE
            stack.append(BVV(mem.size, 256))
        elif op == 0x5B:                             # JUMPDEST
            pass
        elif op == 0xF3:                             # RETURN
            _pop(stack), _pop(stack)
            return result("return")
        elif op == 0xFF:                             # SELFDESTRUCT :1823-1845 (ends the call; storage kept)
            _pop(stack)
            return result("selfdestruct")
        elif op == 0xFE:
            raise ExceptionalHalt("invalid opcode")
        else:
            raise ReplayUnsupported(f"opcode 0x{op:02x}")
        if len(stack) > 1024:
            raise ExceptionalHalt("stack overflow")


def replay_assignment(vec: dict):
    """Concrete coordinates of a VMTests-style request (hex strings as in the JSON)."""
    data = bytes.fromhex(vec.get("data", ""))
    scal = {
        "caller": int(vec["caller"], 16),
        "origin": int(vec["origin"], 16),
        "address": int(vec["address"], 16),
        "callvalue": int(vec["value"], 16),
        "gasprice": int(vec["gasPrice"], 16),
        "calldatasize": len(data),
    }
    arrays = {"calldata": ({i: b for i, b in enumerate(data)}, 0)}
    return scal, arrays


def engine_follow(engine, scal: Dict[str, int], arrays=None):
    """``follow`` for :func:`replay` through the product path: the decision term evaluated on the
    GPU (``mg_eval``) under the request's concrete inputs — scalar coordinates by name, array sites
    (``calldata[...]``) by the concrete byte at their key (the key itself evaluated the same way)."""
    from . import ssa

    arrays = arrays or {}

    def value(term: T.Term) -> int:
        P = ssa.flatten([T.BoolVal(True), T.eq(term, term)], extra=[term])
        P.set_watch([P.term_node[term.id]])
        assign = []
        for c in P.coords:
            if c.kind == ssa.COORD_SCALAR:
                assign.append(scal.get(c.name, 0))
            else:
                assign.append(None)
        for c in P.sites:  # a site's key is a term over the inputs: evaluate it first
            key = value(P.node_term[P.site_key_node[c.index]])
            table, dflt = arrays.get(c.name, ({}, 0))
            assign[c.index] = table.get(key, dflt)
        soa = ssa.soa_from_assignments(P, [assign])
        prog = engine.load(P.to_bytes())
        try:
            info = engine.info(prog)
            _, watch = engine.eval(prog, soa, 1, watch_words=info.watch_words)
        finally:
            engine.free(prog)
        return ssa.limbs_to_int(watch[:, 0])

    return value
