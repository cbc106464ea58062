"""Mirror of LASER's ``KeccakFunctionManager`` over the engine's term mirror.

Same construction as ``mythril/laser/ethereum/keccak_function_manager.py:24-152``:
symbolic SHA3 input of N bits becomes ``keccak256_N(data)`` (an uninterpreted
function) plus the side condition

    inv(f(x)) == x  and  ( lo <= f(x) < lo + PART  and  f(x) % 64 == 0
                           or  OR over known concrete hashes (f(x) == h and x == k) )

where the interval index of each input width is handed out in first-seen order
(``:17-19, 129-137``).  Concrete input data is hashed for real — on the GPU
(``mg_keccak256``) instead of ``ethereum.utils.sha3`` (``:44-57``).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

from .smt import (And, BitVec, Bool, Function, Or, ULE, ULT, URem, symbol_factory)

TOTAL_PARTS = 10 ** 40
PART = (2 ** 256 - 1) // TOTAL_PARTS
INTERVAL_DIFFERENCE = 10 ** 30
EMPTY_KECCAK = 89477152217924674838424037953991966239322087453347756267410168184682657981552


class KeccakFunctionManager:
    def __init__(self, hasher=None):
        self.store_function: Dict[int, Tuple[Function, Function]] = {}
        self.interval_hook_for_size: Dict[int, int] = {}
        self._index_counter = TOTAL_PARTS - 34534
        self.hash_result_store: Dict[int, List[BitVec]] = {}
        self.concrete_hashes: Dict[BitVec, BitVec] = {}
        self._hasher = hasher

    def find_concrete_keccak(self, data: BitVec) -> BitVec:
        if self._hasher is None:
            from .native import Engine

            self._hasher = lambda msgs: Engine.get().keccak256(msgs)
        digest = self._hasher([data.value.to_bytes(data.size() // 8, "big")])[0]
        return symbol_factory.BitVecVal(int.from_bytes(digest, "big"), 256)

    def get_function(self, length: int) -> Tuple[Function, Function]:
        try:
            return self.store_function[length]
        except KeyError:
            func = Function("keccak256_{}".format(length), length, 256)
            inverse = Function("keccak256_{}-1".format(length), 256, length)
            self.store_function[length] = (func, inverse)
            self.hash_result_store[length] = []
            return func, inverse

    @staticmethod
    def get_empty_keccak_hash() -> BitVec:
        return symbol_factory.BitVecVal(EMPTY_KECCAK, 256)

    def interval(self, length: int) -> Tuple[int, int]:
        try:
            index = self.interval_hook_for_size[length]
        except KeyError:
            self.interval_hook_for_size[length] = self._index_counter
            index = self._index_counter
            self._index_counter -= INTERVAL_DIFFERENCE
        lower = index * PART
        return lower, lower + PART

    def create_keccak(self, data: BitVec) -> Tuple[BitVec, Bool]:
        length = data.size()
        func, inverse = self.get_function(length)
        if data.symbolic is False:
            concrete_hash = self.find_concrete_keccak(data)
            self.concrete_hashes[data] = concrete_hash
            condition = And(func(data) == concrete_hash, inverse(func(data)) == data)
            return concrete_hash, condition
        condition = self._create_condition(func_input=data)
        self.hash_result_store[length].append(func(data))
        return func(data), condition

    def _create_condition(self, func_input: BitVec) -> Bool:
        length = func_input.size()
        func, inv = self.get_function(length)
        lower, upper = self.interval(length)
        cond = And(
            inv(func(func_input)) == func_input,
            ULE(symbol_factory.BitVecVal(lower, 256), func(func_input)),
            ULT(func(func_input), symbol_factory.BitVecVal(upper, 256)),
            URem(func(func_input), symbol_factory.BitVecVal(64, 256)) == 0,
        )
        concrete_cond = symbol_factory.Bool(False)
        for key, keccak in self.concrete_hashes.items():
            hash_eq = And(func(func_input) == keccak, key == func_input)
            concrete_cond = Or(concrete_cond, hash_eq)
        return And(inv(func(func_input)) == func_input, Or(cond, concrete_cond))
