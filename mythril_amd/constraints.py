"""Mirror of LASER's ``Constraints`` (``mythril/laser/ethereum/state/constraints.py:9-121``)
over the engine's ``get_model``.

``is_possible`` is the reachability prune LASER runs for every successor
state (``svm.py:252-257``): here it is one GPU search
(``solver.get_model``), True when a model is found and False on
``UnsatError``, which the engine raises when the budget runs out without a
model (inside Mythril the hook would have fallen through to z3 instead).
Successor states share this list's prefix, so the search's flattening cache
(``ssa.FlattenCache``) re-flattens only the appended condition.
"""
from __future__ import annotations

from typing import Iterable, List, Optional, Union

from . import solver
from .smt import Bool, simplify, symbol_factory


class Constraints(list):
    def __init__(self, constraint_list: Optional[List[Union[bool, Bool]]] = None) -> None:
        super().__init__(self._get_smt_bool_list(constraint_list or []))

    @property
    def is_possible(self) -> bool:
        try:
            solver.get_model(tuple(self[:]))
        except solver.UnsatError:
            return False
        return True

    def append(self, constraint: Union[bool, Bool]) -> None:
        # constraints.py:37-45: Bool terms are simplified, Python bools wrapped
        constraint = simplify(constraint) if isinstance(constraint, Bool) else symbol_factory.Bool(constraint)
        super().append(constraint)

    def pop(self, index: int = -1) -> None:
        raise NotImplementedError  # constraints.py:47-53

    @property
    def as_list(self) -> List[Bool]:
        return self[:]

    def __copy__(self) -> "Constraints":
        return Constraints(super().copy())

    def copy(self) -> "Constraints":
        return self.__copy__()

    def __deepcopy__(self, memodict=None) -> "Constraints":
        return self.__copy__()

    def __add__(self, constraints: List[Union[bool, Bool]]) -> "Constraints":
        return Constraints(constraint_list=super().__add__(self._get_smt_bool_list(constraints)))

    def __iadd__(self, constraints: Iterable[Union[bool, Bool]]) -> "Constraints":
        super().__iadd__(self._get_smt_bool_list(constraints))
        return self

    @staticmethod
    def _get_smt_bool_list(constraints: Iterable[Union[bool, Bool]]) -> List[Bool]:
        return [c if isinstance(c, Bool) else symbol_factory.Bool(c) for c in constraints]

    def __hash__(self):
        return tuple(self[:]).__hash__()
