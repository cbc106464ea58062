"""Host-side replacement of interval hashes by real Keccak-256 in printed
transactions (``mythril/analysis/solver.py:119-152``) and
``get_concrete_hash_data`` (``keccak_function_manager.py:103-119``).
CPU tests drive the host logic with the oracle as evaluator and hasher; the GPU
test runs the product path (``Model.eval_many`` + ``mg_keccak256``)."""
import pytest

from mythril_amd.keccak_model import KeccakFunctionManager, hash_matcher, replace_with_actual_sha
from mythril_amd.smt import symbol_factory
from oracle.bv import OracleModel, evaluate
from oracle.keccak import keccak256 as oracle_keccak

BVS = symbol_factory.BitVecSym


class _V(int):
    def as_long(self):
        return int(self)


def _setup():
    km = KeccakFunctionManager(hasher=lambda msgs: [oracle_keccak(m) for m in msgs])
    a = BVS("a", 256)
    h, _ = km.create_keccak(a)
    lo, _ = km.interval(256)
    a_val, h_val = 0x1234, lo + 64 * 5
    funcs = {"keccak256_256": ({a_val: h_val}, 0), "keccak256_256-1": ({h_val: a_val}, 0)}
    model = OracleModel({"a": a_val}, {}, funcs)
    ev = lambda terms: [_V(evaluate(t, model)) for t in terms]  # noqa: E731
    return km, h_val, a_val, ev, funcs


def test_interval_hash_prints_with_matcher():
    km, h_val, _, _, _ = _setup()
    assert hash_matcher in "%064x" % h_val


def test_get_concrete_hash_data():
    km, h_val, _, ev, _ = _setup()
    assert km.get_concrete_hash_data(None, ev) == {256: [h_val]}


def test_replace_with_actual_sha():
    km, h_val, a_val, ev, _ = _setup()
    real = oracle_keccak(a_val.to_bytes(32, "big")).hex()
    txs = [{"input": "0xa9059cbb" + "%064x" % h_val + "00" * 32},
           {"input": "0xa9059cbb" + "11" * 32}]
    replace_with_actual_sha(txs, None, km, evaluate=ev)
    assert txs[0]["input"] == "0xa9059cbb" + real + "00" * 32
    assert txs[1]["input"] == "0xa9059cbb" + "11" * 32


def test_unknown_hash_left_alone():
    km, h_val, _, ev, _ = _setup()
    other = "%064x" % (h_val + 64)  # in the interval, but not a stored hash value
    txs = [{"input": "0xa9059cbb" + other}]
    replace_with_actual_sha(txs, None, km, evaluate=ev)
    assert txs[0]["input"] == "0xa9059cbb" + other


@pytest.mark.gpu
def test_replace_with_actual_sha_on_gpu(engine):
    from mythril_amd.solver import Model

    km, h_val, a_val, _, funcs = _setup()
    km._hasher = None  # product hasher: mg_keccak256
    model = Model({"a": a_val}, {}, funcs)
    assert km.get_concrete_hash_data(model) == {256: [h_val]}
    txs = [{"input": "0xa9059cbb" + "%064x" % h_val}]
    replace_with_actual_sha(txs, model, km)
    assert txs[0]["input"] == "0xa9059cbb" + oracle_keccak(a_val.to_bytes(32, "big")).hex()


@pytest.mark.gpu
def test_engine_calls_from_two_threads(engine):
    """The z3 race's thread layout: a search on one worker thread while another
    thread hashes through ``mg_keccak256`` — neither thread ran ``mg_init``, and every entry
    point makes the engine's device current on its calling thread (``OnDevice``)."""
    import threading

    from mythril_amd import search, workloads

    roots = [c.raw for c in workloads.WORKLOADS["token_transfer_underflow"]()]
    out = {}

    def hashing():
        msgs = [bytes([k]) * k for k in range(1, 40)]
        out["k"] = (engine.keccak256(msgs), [oracle_keccak(m) for m in msgs])

    def searching():
        out["s"] = search.search(engine, roots, jit="never", timeout_s=5)

    ts = [threading.Thread(target=hashing), threading.Thread(target=searching)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    got, want = out["k"]
    assert [bytes(g) for g in got] == want
    assert out["s"].index is not None
