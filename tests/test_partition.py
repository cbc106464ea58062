"""Independence partitioning (host logic, CPU), after the reference's
tests/laser/smt/independece_solver_test.py."""
import random

from mythril_amd.keccak_model import KeccakFunctionManager
from mythril_amd.partition import DependenceMap, get_expr_variables, partition
from mythril_amd.smt import Array, If, UGT, symbol_factory
from mythril_amd.smt import terms as T

BVS = symbol_factory.BitVecSym
BVV = symbol_factory.BitVecVal


def test_get_expr_variables():
    x = symbol_factory.BoolSym("x")
    y, z, b = BVS("y", 256), BVS("z", 256), BVS("b", 256)
    assert set(get_expr_variables(If(x, y, z + b).raw)) == {"x", "y", "z", "b"}


def test_get_expr_variables_num():
    b = BVS("b", 256)
    assert get_expr_variables((b + BVV(2, 256)).raw) == ["b"]


def test_dependence_map():
    x, y, z, a, b = (BVS(n, 256) for n in "xyzab")
    conditions = [UGT(x, y).raw, (y == z).raw, (a == b).raw]
    dm = DependenceMap()
    for c in conditions:
        dm.add_condition(c)
    assert len(dm.buckets) == 2
    assert {n for _, n in dm.buckets[0].variables} == {"x", "y", "z"}
    assert dm.buckets[0].conditions == conditions[:2]
    assert {n for _, n in dm.buckets[1].variables} == {"a", "b"}
    assert dm.buckets[1].conditions == conditions[2:]


def test_merge_keeps_input_order():
    x, y, z = (BVS(n, 256) for n in "xyz")
    cs = [(x == BVV(1, 256)).raw, (y == BVV(2, 256)).raw, (x == y).raw, (z == BVV(0, 256)).raw]
    assert partition(cs) == [cs[:3], cs[3:]]


def test_arrays_and_ground_conditions():
    st = Array("Storage", 256, 256)
    x, y = BVS("x", 256), BVS("y", 256)
    g = T.BoolVal(True)
    cs = [(st[x] == BVV(1, 256)).raw, g, (st[y] == BVV(2, 256)).raw, (x == BVV(3, 256)).raw]
    # one shared array couples every condition that reads it
    assert partition(cs) == [[g], [cs[0], cs[2], cs[3]]]


def test_keccak_and_inverse_stay_together():
    km = KeccakFunctionManager()
    a, b = BVS("a", 256), BVS("b", 256)
    o1, c1 = km.create_keccak(a)
    o2, c2 = km.create_keccak(b)
    buckets = partition([c1.raw, c2.raw, (o1 == BVV(5, 256)).raw])
    # both applications use the same keccak256_256 / keccak256_256-1 pair
    assert len(buckets) == 1


def test_random_partitions_are_disjoint_and_complete():
    rng = random.Random(7)
    names = [f"v{i}" for i in range(12)]
    for _ in range(50):
        cs = []
        for _ in range(rng.randint(1, 10)):
            k = rng.sample(names, rng.randint(1, 3))
            t = BVS(k[0], 64)
            for n in k[1:]:
                t = t + BVS(n, 64)
            cs.append((t == BVV(rng.getrandbits(64), 64)).raw)
        buckets = partition(cs)
        assert sorted(c.id for b in buckets for c in b) == sorted({c.id for c in cs})
        seen = set()
        for b in buckets:
            vs = set().union(*(set(get_expr_variables(c)) for c in b))
            assert not (vs & seen)
            seen |= vs
