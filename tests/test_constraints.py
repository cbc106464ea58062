"""``Constraints`` mirror (``laser/ethereum/state/constraints.py``): list
behaviour on CPU, ``is_possible`` (one GPU search) on the GPU."""
import copy

import pytest

from mythril_amd import solver
from mythril_amd.constraints import Constraints
from mythril_amd.smt import Bool, symbol_factory

BVS = symbol_factory.BitVecSym
BVV = symbol_factory.BitVecVal


def test_python_bools_are_wrapped_and_terms_simplified():
    x = BVS("x", 256)
    c = Constraints([True])
    c.append(BVV(2, 256) + BVV(3, 256) == BVV(5, 256))  # folds to a literal True
    c.append(x == BVV(1, 256))
    assert all(isinstance(k, Bool) for k in c)
    assert c[1].is_true and not c[2].is_true


def test_copy_add_iadd_keep_type_and_share_prefix():
    x = BVS("x", 256)
    a = Constraints([x == BVV(1, 256)])
    b = copy.copy(a)
    b.append(x != BVV(2, 256))
    assert type(b) is Constraints and len(a) == 1 and len(b) == 2
    assert b[0] is a[0]  # successor states share the parent's terms (prefix reuse)
    c = a + [False]
    assert type(c) is Constraints and c[1].is_false
    a += [True]
    assert len(a) == 2 and a.as_list == a[:]
    assert copy.deepcopy(a) == a[:] and type(copy.deepcopy(a)) is Constraints


def test_pop_is_not_supported():
    with pytest.raises(NotImplementedError):
        Constraints().pop()


def test_hash_is_the_tuple_hash():
    x = BVS("x", 256)
    c = Constraints([x == BVV(1, 256)])
    assert hash(c) == hash(tuple(c))


@pytest.mark.gpu
def test_is_possible(engine):
    x = BVS("x", 256)
    c = Constraints([x == BVV(5, 256)])
    assert c.is_possible
    old = solver.args.solver_timeout
    solver.args.solver_timeout = 300
    try:
        d = c + [x == BVV(6, 256)]
        assert not d.is_possible
        assert not Constraints([False]).is_possible
    finally:
        solver.args.solver_timeout = old
