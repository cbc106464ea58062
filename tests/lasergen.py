"""Random LASER-shaped queries for differential tests of the compiled tiers (test infrastructure).

``laser_query(seed)`` composes a ``get_model`` query the way LASER builds them for token-style
contracts, from the same emitters ``mythril_amd/workloads.py`` follows (each cited there):
transaction symbols and the solc dispatcher, the actor disjunction, keccak-keyed mappings with
their side conditions (``keccak_function_manager.py:83-149``: the inverse-map lookups with one
prior per earlier site, literal-slot tails), Store chains read back through Select, the integer
module's wrap predicates, ITE guards, equalities between symbols (so the generator's MIXED
coordinates copy one another in chains), and random arithmetic over the words it has built.
``full=True`` adds the vocabulary outside the first tier's original set: symbolic divisors
(``instructions.py:480-566``), symbolic shift amounts (``:528-552``), EXP (``:599-631``) and
concrete Keccak-256 of data (``keccak_function_manager.py:44-57``).
"""
from __future__ import annotations

import random
from typing import List

from mythril_amd import workloads as W
from mythril_amd.keccak_model import KeccakFunctionManager
from mythril_amd.smt import (Array, BitVec, BVAddNoOverflow, BVMulNoOverflow, BVSubNoUnderflow, Concat, Extract, If,
                             LShR, Not, Or, SRem, UDiv, UGE, UGT, ULE, ULT, URem, simplify, symbol_factory)
from mythril_amd.smt import terms as T

BVV = symbol_factory.BitVecVal
BVS = symbol_factory.BitVecSym
M160 = BVV(W.MASK160, 256)


def _lit(rng: random.Random) -> int:
    return rng.choice([0, 1, 2, 3, 20, 255, 256, 2300, 604800, 86400, 10 ** 18, (1 << 160) - 1, (1 << 255),
                       (1 << 256) - 1, (1 << 256) - 2, rng.getrandbits(rng.choice([8, 32, 64, 160, 256]))])


def laser_query(seed: int, full: bool = False, max_tx: int = 3) -> List:
    rng = random.Random(seed)
    km = KeccakFunctionManager()
    storage = Array("Storage", 256, 256)
    conds = []
    words = []   # 256-bit terms to combine
    n_tx = rng.randint(1, max_tx)
    for tid in range(1, n_tx + 1):
        tx = W.Tx(tid)
        n_args = rng.randint(1, 3)
        if rng.random() < 0.85:
            d = tx.dispatch(rng.choice(list(W.SELECTORS.values())), n_args)
            conds += [c for c in d if rng.random() < 0.8]
        elif rng.random() < 0.5:
            conds.append(tx.actor())
        args = [tx.arg(k) for k in range(n_args)]
        sender = tx.sender & M160
        words += args + [tx.sender, tx.value]
        if rng.random() < 0.3:
            words.append(tx.size)
        # mappings: balance[key] at a literal slot, read, sometimes written back (Store chains)
        for _ in range(rng.randint(0, 3)):
            key = rng.choice([sender, args[0] & M160, args[-1], rng.choice(words)])
            slot = rng.choice([0, 1, 2, 3, W.W_OWNER_INDEX, W.W_PENDING])
            k = W.mapping_slot(km, key, slot, conds)
            bal = storage[k] if rng.random() < 0.5 else simplify(storage[k])
            words.append(bal)
            if rng.random() < 0.5:
                storage[k] = rng.choice([bal - args[-1], bal + args[-1], BVV(_lit(rng), 256), rng.choice(words)])
        if rng.random() < 0.3:  # a mapping keyed by a keccak of calldata bytes (keccak256_288-style UF)
            nb = rng.choice([4, 36])
            k = W.mapping_slot_raw(km, Concat([tx.byte(q) for q in range(nb)]), conds)
            words.append(storage[k])
        for _ in range(rng.randint(0, 2)):  # plain slots
            s = BVV(rng.randint(0, 5), 256)
            if rng.random() < 0.5:
                storage[s] = rng.choice(words)
            words.append(storage[s])
        if rng.random() < 0.3:
            conds.append(tx.sender == BVV(rng.choice([W.ATTACKER, W.CREATOR, W.SOMEGUY]), 256))
        if rng.random() < 0.2:
            conds.append(tx.sender == BVS(f"origin{tid}", 256))
    if rng.random() < 0.3:
        words.append(BVS("timestamp", 256))
    # predicates over the words (the detection modules' and the path's)
    for _ in range(rng.randint(2, 7)):
        a, b = rng.choice(words), rng.choice(words)
        lit = BVV(_lit(rng), 256)
        kind = rng.randrange(16 if not full else 22)
        if kind == 0:
            p = UGE(a, b)
        elif kind == 1:
            p = ULT(a, rng.choice([b, lit]))
        elif kind == 2:
            p = ULE(a, lit)
        elif kind == 3:
            p = UGT(a, lit)
        elif kind == 4:
            p = a == b
        elif kind == 5:
            p = Not(a == rng.choice([b, lit]))
        elif kind == 6:
            p = Not(BVSubNoUnderflow(a, b, False))
        elif kind == 7:
            p = Not(BVMulNoOverflow(a, rng.choice([b, BVS("cnt", 256)]), False))
        elif kind == 8:
            p = Not(BVAddNoOverflow(a, b, False))
        elif kind == 9:
            p = ULT(a + b, a)
        elif kind == 10:
            p = If(a == lit, b, a + BVV(1, 256)) == rng.choice(words)
        elif kind == 11:
            p = a < rng.choice([b, lit])  # signed (z3py '<')
        elif kind == 12:
            p = (a & BVV((1 << rng.choice([8, 32, 160])) - 1, 256)) == (lit & BVV(0xFFFFFFFF, 256))
        elif kind == 13:
            p = UGE(UDiv(a, BVV(rng.choice([3, 10, 86400, 10 ** 9, 1 << 224]), 256)), BVV(rng.randint(0, 5), 256))
        elif kind == 14:
            p = URem(a, BVV(rng.choice([2, 64, 1000, 7]), 256)) == BVV(0, 256)
        elif kind == 15:
            p = Or(UGT(a, BVV(16, 256)), a == BVV(0, 256))
        elif kind == 16:
            p = ULT(UDiv(a, b), lit)
        elif kind == 17:
            p = URem(a, b) == BVV(rng.randint(0, 3), 256)
        elif kind == 18:
            p = (a / rng.choice([b, lit])) < (b % lit)  # SDIV / SMOD (z3py operators)
        elif kind == 19:
            sh = b & BVV(rng.choice([0xFF, 0x1FF, 7]), 256)
            p = rng.choice([LShR(a, sh), a << sh, a >> sh]) == rng.choice([lit, b])
        elif kind == 20:
            e = BitVec(T.bvexp(rng.choice([a, BVV(rng.choice([2, 10, 256]), 256)]).raw, (b & BVV(0xFF, 256)).raw))
            p = ULT(e, rng.choice([lit, a]))
        else:
            h = BitVec(T.keccak256(Concat(a & M160, BVV(rng.randint(0, 3), 256)).raw))
            p = ULT(h, BVV(1 << rng.choice([240, 250, 255]), 256)) if rng.random() < 0.5 else \
                Not(h == SRem(b, lit))
        conds.append(p)
    if rng.random() < 0.3:
        e = rng.randrange(len(conds))
        conds[e] = Not(conds[e])
    if rng.random() < 0.3:
        w = rng.choice(words)
        conds.append(ULT(Extract(63, 0, w), BVV(rng.getrandbits(64), 64)))
    rng.shuffle(conds)
    return [c.raw for c in conds]
