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

hash_matcher = "fffffff"  # keccak_function_manager.py:20: prefix of interval hashes in printed inputs
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

    def _hash(self, msgs: List[bytes]) -> List[bytes]:
        if self._hasher is None:
            from .native import Engine

            self._hasher = lambda m: Engine.get().keccak256(m)
        return self._hasher(msgs)

    def find_concrete_keccak(self, data: BitVec) -> BitVec:
        digest = self._hash([data.value.to_bytes(data.size() // 8, "big")])[0]
        return symbol_factory.BitVecVal(int.from_bytes(digest, "big"), 256)

    def find_concrete_keccaks(self, datas: List[BitVec]) -> List[BitVec]:
        """Batched :meth:`find_concrete_keccak`: one ``mg_keccak256`` launch for all inputs."""
        digests = self._hash([d.value.to_bytes(d.size() // 8, "big") for d in datas])
        return [symbol_factory.BitVecVal(int.from_bytes(h, "big"), 256) for h in digests]

    def get_concrete_hash_data(self, model, evaluate=None) -> Dict[int, List[int]]:
        """``keccak_function_manager.py:103-119``: concrete values of every stored
        symbolic hash under ``model``, evaluated in one batch (``Model.eval_many``);
        values that stay symbolic are skipped, as the reference's ``as_long``
        AttributeError branch does."""
        evaluate = evaluate or (lambda terms: model.eval_many(terms, model_completion=False))
        sizes = list(self.hash_result_store)
        flat = [v.raw for size in sizes for v in self.hash_result_store[size]]
        vals = iter(evaluate(flat) if flat else [])
        out: Dict[int, List[int]] = {}
        for size in sizes:
            out[size] = []
            for _ in self.hash_result_store[size]:
                v = next(vals)
                if hasattr(v, "as_long"):
                    out[size].append(v.as_long())
        return out

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


def replace_with_actual_sha(concrete_transactions: List[Dict[str, str]], model, km: KeccakFunctionManager,
                            code=None, evaluate=None, bvv=None) -> None:
    """``mythril/analysis/solver.py:119-152`` on the engine: every 64-hex-digit
    slice of a printed transaction input that is a stored interval hash (it
    contains ``hash_matcher``) is replaced by the real Keccak-256 of its
    preimage ``inverse(hash)`` under ``model``.

    Same scan and the same in-place, left-to-right replacements as the reference.
    The preimages of the slices of the unmodified inputs are evaluated in one
    batch and hashed in one ``mg_keccak256`` launch up front; a slice that only
    appears after an earlier replacement is evaluated and hashed on demand."""
    evaluate = evaluate or (lambda terms: model.eval_many(terms, model_completion=False))
    bvv = bvv or symbol_factory.BitVecVal  # LASER's factory when driving LASER's manager
    concrete_hashes = km.get_concrete_hash_data(model, evaluate)
    bytecode = getattr(code, "bytecode", None)

    def s_index_of(tx):
        return len(bytecode) + 2 if bytecode is not None and bytecode in tx["input"] else 10

    def preimages(words: List[int]) -> Dict[int, BitVec]:
        todo, keys = [], []
        for w in words:
            for size in concrete_hashes:
                if w in concrete_hashes[size]:  # the reference keeps the LAST matching size
                    _, inverse = km.store_function[size]
                    todo.append(inverse(bvv(w, 256)).raw)
                    keys.append((w, size))
        res: Dict[int, BitVec] = {}
        for (w, size), v in zip(keys, evaluate(todo) if todo else []):
            res[w] = bvv(v.as_long(), size)
        return res

    def scan(inp: str, s_index: int) -> List[int]:
        out = []
        for i in range(s_index, len(inp)):
            sl = inp[i:i + 64]
            if hash_matcher in sl and len(sl) == 64:
                out.append(int(sl, 16))
        return out

    words = sorted({w for tx in concrete_transactions if hash_matcher in tx["input"]
                    for w in scan(tx["input"], s_index_of(tx))})
    pre = preimages(words)
    keys = sorted(pre)
    digests = dict(zip(keys, (k.value for k in km.find_concrete_keccaks([pre[k] for k in keys])))) if keys else {}

    for tx in concrete_transactions:
        if hash_matcher not in tx["input"]:
            continue
        s_index = s_index_of(tx)
        for i in range(s_index, len(tx["input"])):
            data_slice = tx["input"][i:i + 64]
            if hash_matcher not in data_slice or len(data_slice) != 64:
                continue
            w = int(data_slice, 16)
            if w not in digests:
                more = preimages([w])
                if w not in more:
                    continue
                pre[w] = more[w]
                digests[w] = km.find_concrete_keccak(more[w]).value
            hex_keccak = "%064x" % digests[w]
            tx["input"] = tx["input"][:s_index] + tx["input"][s_index:].replace(tx["input"][i:64 + i], hex_keccak)
