"""Synthetic LASER queries for the configurations named in BASELINE.json.

There is no solc and no z3 in this image, so the ``get_model`` queries of
``myth analyze`` cannot be dumped here.  These builders construct the same
constraint *shapes* LASER emits for the named contracts, term by term through
the ``mythril.laser.smt`` mirror, following the emitters cited inline:

* transaction symbols  ``sender_<tx>``, ``call_value<tx>``, ``<tx>_calldatasize``,
  ``<tx>_calldata`` (``transaction/symbolic.py:87-104``, ``calldata.py:207-231``);
* actor disjunction    ``Or(sender == CREATOR | ATTACKER | SOMEGUY)``
  (``transaction/symbolic.py:165-167``);
* solc 0.5 dispatcher  ``CALLDATASIZE < 4`` / ``DIV(CALLDATALOAD(0), 2^224) & 0xffffffff == sel``
  (``instructions.py:480-494, 666-675, 716-740``), nonpayable ``ISZERO(CALLVALUE)``;
* mappings             ``Storage[keccak256_512(pad(key) ++ slot)]`` with the keccak side condition
  (``keccak_function_manager.py:83-149``, ``account.py:62``);
* detection predicates ``Not(BVSubNoUnderflow)``, ``Not(BVMulNoOverflow)`` (``integer.py:141-160``),
  reentrancy ``UGT(gas, 2300)`` (``state_change_external_calls.py:53,132``).
"""
from __future__ import annotations

from typing import List

from .keccak_model import KeccakFunctionManager
from .smt import (And, Array, BVMulNoOverflow, BVSubNoUnderflow, Bool, Concat, If, Not, Or, UDiv, UGE, UGT, ULE,
                  ULT, symbol_factory)

BVV = symbol_factory.BitVecVal
BVS = symbol_factory.BitVecSym

CREATOR = 0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE
ATTACKER = 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF
SOMEGUY = 0xAAAAAAAABBBBBBBBCCCCCCCCDDDDDDDDEEEEEEEE

# keccak256 of the Solidity signatures (pinned against oracle/keccak.py by tests)
SEL_TRANSFER = 0xA9059CBB          # transfer(address,uint256)
SEL_WITHDRAW = 0x155DD5EE          # withdrawFunds(uint256)
SEL_BATCH_TRANSFER = 0x83F12FEC    # batchTransfer(address[],uint256)
SELECTORS = {
    "transfer(address,uint256)": SEL_TRANSFER,
    "withdrawFunds(uint256)": SEL_WITHDRAW,
    "batchTransfer(address[],uint256)": SEL_BATCH_TRANSFER,
}
MASK160 = (1 << 160) - 1


class Tx:
    """Symbols of one symbolic message call."""

    def __init__(self, tx_id: int):
        self.id = tx_id
        self.calldata = Array(f"{tx_id}_calldata", 256, 8)
        self.size = BVS(f"{tx_id}_calldatasize", 256)
        self.sender = BVS(f"sender_{tx_id}", 256)
        self.value = BVS(f"call_value{tx_id}", 256)

    def byte(self, i: int):
        # SymbolicCalldata._load (calldata.py:217-231): If(item < size, calldata[item], 0), signed '<'
        item = BVV(i, 256)
        return If(item < self.size, self.calldata[item], BVV(0, 8))

    def word(self, off: int):
        return Concat([self.byte(off + k) for k in range(32)])

    def actor(self) -> Bool:
        return Or(self.sender == BVV(CREATOR, 256), self.sender == BVV(ATTACKER, 256),
                  self.sender == BVV(SOMEGUY, 256))

    def dispatch(self, selector: int, n_args: int) -> List[Bool]:
        sel = UDiv(self.word(0), BVV(1 << 224, 256)) & BVV(0xFFFFFFFF, 256)
        return [
            self.actor(),
            Not(ULT(self.size, BVV(4, 256))),
            sel == BVV(selector, 256),
            If(self.value == 0, BVV(1, 256), BVV(0, 256)) != 0,      # nonpayable: ISZERO(CALLVALUE)
            If(ULT(self.size - 4, BVV(32 * n_args, 256)), BVV(1, 256), BVV(0, 256)) == 0,  # abi length check
        ]

    def arg(self, k: int):
        return self.word(4 + 32 * k)


def mapping_slot(km: KeccakFunctionManager, key, slot: int, conds: List[Bool]):
    """``mapping[key]`` storage index: keccak256(pad32(key) ++ slot) and its side condition."""
    data = Concat(key, BVV(slot, 256))
    h, c = km.create_keccak(data)
    conds.append(c)
    return h


def token_transfer_underflow() -> List[Bool]:
    """C2 (token.sol ``transfer``, -t 2): tx 1 transfers, tx 2's
    ``balances[msg.sender] -= _value`` can underflow (integer module, SWC-101)."""
    km = KeccakFunctionManager()
    storage = Array("Storage", 256, 256)
    conds: List[Bool] = []
    txs = [Tx(1), Tx(2)]
    for tx in txs:
        conds += tx.dispatch(SEL_TRANSFER, 2)
        to = tx.arg(0) & BVV(MASK160, 256)
        value = tx.arg(1)
        k_from = mapping_slot(km, tx.sender & BVV(MASK160, 256), 0, conds)
        bal_from = storage[k_from]
        if tx.id == 2:
            conds.append(Not(BVSubNoUnderflow(bal_from, value, False)))
            break
        storage[k_from] = bal_from - value
        k_to = mapping_slot(km, to, 0, conds)
        storage[k_to] = storage[k_to] + value
    return conds


def etherstore_reentrancy() -> List[Bool]:
    """C2 (etherstore.sol ``withdrawFunds``): the external call after the checks is
    reachable with > 2300 gas (state_change_external_calls)."""
    km = KeccakFunctionManager()
    storage = Array("Storage", 256, 256)
    conds: List[Bool] = []
    tx = Tx(2)
    conds += tx.dispatch(SEL_WITHDRAW, 1)
    w = tx.arg(0)
    sender = tx.sender & BVV(MASK160, 256)
    bal = storage[mapping_slot(km, sender, 2, conds)]
    last = storage[mapping_slot(km, sender, 1, conds)]
    limit = storage[BVV(0, 256)]
    now = BVS("timestamp", 256)
    gas = BVS(f"{tx.id}_gas", 256)
    conds += [
        UGE(bal, w),
        ULE(w, limit),
        UGE(now, last + BVV(604800, 256)),
        UGT(gas, BVV(2300, 256)),
        Or(UGT(sender, BVV(16, 256)), sender == 0),
    ]
    return conds


def bectoken_batch_overflow() -> List[Bool]:
    """C3 (BECToken.sol ``batchTransfer``): ``amount = cnt * _value`` overflows
    (integer module BVMulNoOverflow) with 0 < cnt <= 20, value > 0 and
    ``balances[msg.sender] >= amount``."""
    km = KeccakFunctionManager()
    storage = Array("Storage", 256, 256)
    conds: List[Bool] = []
    tx = Tx(1)
    conds += tx.dispatch(SEL_BATCH_TRANSFER, 2)
    value = tx.arg(1)
    cnt = BVS("receivers_len", 256)  # length of the dynamic array (read via calldata offset)
    amount = cnt * value
    bal = storage[mapping_slot(km, tx.sender & BVV(MASK160, 256), 0, conds)]
    conds += [
        Not(BVMulNoOverflow(cnt, value, False)),
        UGT(cnt, BVV(0, 256)),
        ULE(cnt, BVV(20, 256)),
        UGT(value, BVV(0, 256)),
        UGE(bal, amount),
    ]
    return conds


WORKLOADS = {
    "token_transfer_underflow": token_transfer_underflow,
    "etherstore_reentrancy": etherstore_reentrancy,
    "bectoken_batch_overflow": bectoken_batch_overflow,
}
