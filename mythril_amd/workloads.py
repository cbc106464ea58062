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
from .smt import (And, Array, BitVec, simplify, BVMulNoOverflow, BVSubNoUnderflow, Bool, Concat, If, Not, Or, UDiv, UGE, UGT,
                  ULE, ULT, symbol_factory)
from .smt import terms as T

BVV = symbol_factory.BitVecVal
BVS = symbol_factory.BitVecSym

CREATOR = 0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE
ATTACKER = 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF
SOMEGUY = 0xAAAAAAAABBBBBBBBCCCCCCCCDDDDDDDDEEEEEEEE

# keccak256 of the Solidity signatures (pinned against oracle/keccak.py by tests)
SEL_TRANSFER = 0xA9059CBB          # transfer(address,uint256)
SEL_WITHDRAW = 0x155DD5EE          # withdrawFunds(uint256)
SEL_BATCH_TRANSFER = 0x83F12FEC    # batchTransfer(address[],uint256)
SEL_INIT_WALLET = 0xE46DCFEB       # initWallet(address[],uint256,uint256)
SEL_CHANGE_REQUIREMENT = 0xBA51A6DF  # changeRequirement(uint256)
SEL_KILL = 0xCBF0B0C0              # kill(address)
SELECTORS = {
    "transfer(address,uint256)": SEL_TRANSFER,
    "withdrawFunds(uint256)": SEL_WITHDRAW,
    "batchTransfer(address[],uint256)": SEL_BATCH_TRANSFER,
    "initWallet(address[],uint256,uint256)": SEL_INIT_WALLET,
    "changeRequirement(uint256)": SEL_CHANGE_REQUIREMENT,
    "kill(address)": SEL_KILL,
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


def suicide_kill() -> List[Bool]:
    """C1 stand-in (``myth analyze solidity_examples/suicide.sol -t 2``; no solc/z3 here, so the
    SURVEY §8(d) fallback shape): tx 1 calls ``kill(addr)`` with ``addr != 0`` (the ``if`` is not
    taken and the call returns), and tx 2 calls ``kill(0)``, which reaches SELFDESTRUCT.  The suicide
    module then asks for a sequence in which every caller is the attacker and the origin
    (``modules/suicide.py:68-81``).  Each symbolic call also carries the balance precondition
    ``UGE(balance[sender], call_value)`` (``transaction/symbolic.py``)."""
    balance = Array("balance", 256, 256)
    conds: List[Bool] = []
    for tx in (Tx(1), Tx(2)):
        conds += tx.dispatch(SEL_KILL, 1)
        addr = tx.arg(0) & BVV(MASK160, 256)
        conds.append(UGE(balance[tx.sender], tx.value))
        conds.append(addr == 0 if tx.id == 2 else addr != 0)
        conds += [tx.sender == BVV(ATTACKER, 256), tx.sender == BVS(f"origin{tx.id}", 256)]
    return conds


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


# WalletLibrary.sol storage slots (solc 0.5 layout of the library's state variables)
W_REQUIRED, W_NUM_OWNERS, W_DAILY_LIMIT, W_LAST_DAY = 0, 1, 2, 4
W_OWNERS = 5                 # uint[256] m_owners
W_OWNER_INDEX = 262          # mapping(uint => uint) m_ownerIndex
W_PENDING = 263              # mapping(bytes32 => PendingState) m_pending (yetNeeded at +0)


def _sload(storage: Array, key):
    """``Storage.__getitem__`` returns ``simplify(storage[item])`` (``account.py:61``)."""
    return simplify(storage[key])


def _confirm_and_check(km: KeccakFunctionManager, tx: Tx, storage: Array, conds: List[Bool]) -> None:
    """``onlymanyowners(keccak256(msg.data))`` → ``confirmAndCheck`` taking the
    "enough confirmations" branch (WalletLibrary.sol:289-313): the sender is an owner,
    and the pending operation's ``yetNeeded`` (reset to ``m_required`` when 0) is <= 1.
    ``keccak256(msg.data)`` of a 36-byte call is the UF ``keccak256_288`` over the
    calldata bytes (``keccak_function_manager.py:83-101``)."""
    conds.append(tx.size == BVV(36, 256))
    op = mapping_slot_raw(km, Concat([tx.byte(k) for k in range(36)]), conds)
    owner_index = _sload(storage, mapping_slot(km, tx.sender & BVV(MASK160, 256), W_OWNER_INDEX, conds))
    conds.append(Not(owner_index == 0))
    pending = _sload(storage, mapping_slot(km, op, W_PENDING, conds))
    yet_needed = If(pending == 0, _sload(storage, BVV(W_REQUIRED, 256)), pending)
    conds.append(ULE(yet_needed, BVV(1, 256)))


def mapping_slot_raw(km: KeccakFunctionManager, data, conds: List[Bool]):
    h, c = km.create_keccak(data)
    conds.append(c)
    return h


def walletlibrary_kill() -> List[Bool]:
    """C4 (WalletLibrary.sol, -t 3): the parity-wallet kill.  tx 1 calls the unprotected
    ``initWallet([owner], required, daylimit)`` (``only_uninitialized``: ``m_numOwners == 0``),
    tx 2 ``changeRequirement(r)`` and tx 3 ``kill(to)`` both pass ``onlymanyowners``; the
    suicide module requires tx 3's caller to be the attacker (``suicide.py``).  Three
    transactions of symbolic calldata, storage written through Store chains at
    keccak-keyed indices, UF keccaks of two input widths (512 and 288 bits).

    The ``address[]`` argument is read at its canonical ABI offset (head word == 0x60), and
    the owner loop takes its one-iteration path, as LASER's JUMPI constraints fix it."""
    km = KeccakFunctionManager()
    storage = Array("Storage", 256, 256)
    conds: List[Bool] = []
    tx1, tx2, tx3 = Tx(1), Tx(2), Tx(3)
    # tx 1: initWallet(address[] _owners, uint _required, uint _daylimit)
    conds += tx1.dispatch(SEL_INIT_WALLET, 3)
    conds.append(_sload(storage, BVV(W_NUM_OWNERS, 256)) == 0)
    conds.append(tx1.arg(0) == BVV(0x60, 256))
    n_owners = tx1.word(4 + 0x60)
    conds += [ULT(BVV(0, 256), n_owners), Not(ULT(BVV(1, 256), n_owners))]
    conds.append(Not(ULT(tx1.size, BVV(4 + 0x60 + 32 + 32, 256))))
    owner0 = tx1.word(4 + 0x60 + 32) & BVV(MASK160, 256)
    sender1 = tx1.sender & BVV(MASK160, 256)
    now = BVS("timestamp", 256)
    storage[BVV(W_DAILY_LIMIT, 256)] = tx1.arg(2)
    storage[BVV(W_LAST_DAY, 256)] = UDiv(now, BVV(86400, 256))
    storage[BVV(W_NUM_OWNERS, 256)] = n_owners + 1
    storage[BVV(W_OWNERS + 1, 256)] = sender1
    storage[mapping_slot(km, sender1, W_OWNER_INDEX, conds)] = BVV(1, 256)
    storage[BVV(W_OWNERS + 2, 256)] = owner0
    storage[mapping_slot(km, owner0, W_OWNER_INDEX, conds)] = BVV(2, 256)
    storage[BVV(W_REQUIRED, 256)] = tx1.arg(1)
    # tx 2: changeRequirement(uint _newRequired) onlymanyowners
    conds += tx2.dispatch(SEL_CHANGE_REQUIREMENT, 1)
    _confirm_and_check(km, tx2, storage, conds)
    new_required = tx2.arg(0)
    conds.append(ULE(new_required, _sload(storage, BVV(W_NUM_OWNERS, 256))))
    storage[BVV(W_REQUIRED, 256)] = new_required
    # tx 3: kill(address _to) onlymanyowners -> selfdestruct, caller is the attacker
    conds += tx3.dispatch(SEL_KILL, 1)
    _confirm_and_check(km, tx3, storage, conds)
    conds.append(tx3.sender == BVV(ATTACKER, 256))
    return conds


def sha3_keyed_mapping() -> List[Bool]:
    """C5 (synthetic SHA3-keyed mapping): concrete Keccak-256 nested
    twice, ``h1 = keccak(pad(a) ++ slot)``, ``h2 = keccak(h1 ++ b)`` (real hashes, as
    LASER computes for concrete data, ``keccak_function_manager.py:44-57``), an EVM
    ``EXP(c, d)`` with an 8-bit exponent and an ``SDIV`` chain (concrete-replay
    semantics, ``instructions.py:497-511, 599-631``).  Predicate:
    ``ULT(h2, 2^240) and SLT(SDIV(x, y), SDIV(EXP(c, d), 3))`` — about 1 candidate in 2^17."""
    a = BVS("a", 256) & BVV(MASK160, 256)
    b, c, x, y = BVS("b", 256), BVS("c", 256), BVS("x", 256), BVS("y", 256)
    d = BVS("d", 256) & BVV(0xFF, 256)
    h1 = BitVec(T.keccak256(Concat(a, BVV(3, 256)).raw))
    h2 = BitVec(T.keccak256(Concat(h1, b).raw))
    e = BitVec(T.bvexp(c.raw, d.raw))
    return [ULT(h2, BVV(1 << 240, 256)), (x / y) < (e / BVV(3, 256))]


WORKLOADS = {
    "suicide_kill": suicide_kill,
    "token_transfer_underflow": token_transfer_underflow,
    "etherstore_reentrancy": etherstore_reentrancy,
    "bectoken_batch_overflow": bectoken_batch_overflow,
    "walletlibrary_kill": walletlibrary_kill,
    "sha3_keyed_mapping": sha3_keyed_mapping,
}

# the BASELINE.json config each workload stands for (``configs[i]`` -> "C{i+1}")
CONFIG = {
    "suicide_kill": "C1",
    "token_transfer_underflow": "C2",
    "etherstore_reentrancy": "C2",
    "bectoken_batch_overflow": "C3",
    "walletlibrary_kill": "C4",
    "sha3_keyed_mapping": "C5",
}


def test_id(name: str) -> str:
    """``C2-token_transfer_underflow``: the config label tests carry in their ids."""
    return f"{CONFIG[name]}-{name}"
