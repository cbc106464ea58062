"""Independence partitioning of a constraint set before the GPU search.

Follows ``mythril/laser/smt/solver/independence_solver.py``: constraints are
grouped into buckets that share no variable (``DependenceMap.add_condition``,
``:45-68``, merging every bucket a new condition touches, ``:70-82``), each
bucket is solved on its own and the bucket models are combined
(``IndependenceSolver.check``/``model``, ``:119-140``).

Why it matters here: the search space of a conjunction is the PRODUCT of its
coordinates' domains, the search space of independent buckets is their SUM.
Two independent 1-in-2^16 conditions cost ~2^32 candidates jointly and ~2^17
when split.

Differences from the reference, all on the side of keeping buckets coupled
where a model could otherwise be inconsistent:

* variables are named symbols — scalars, arrays and uninterpreted functions
  (``_get_expr_variables``, ``:10-22``, takes every childless non-numeral, i.e.
  the same set for scalars and arrays; it never sees a function symbol, so a
  shared UF would not couple buckets there);
* a keccak UF ``keccak256_<n>`` and its inverse ``keccak256_<n>-1``
  (``keccak_function_manager.py:30-33``) count as ONE symbol: the flattener
  defaults the inverse of ``f(x)`` to ``x`` (``ssa.py``), which needs both
  applications in the same program;
* variable-free constraints form one bucket of their own (evaluated once).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

from .smt import terms as T


def get_expr_variables(t: T.Term) -> List[str]:
    """Names of the variables (scalars, arrays, functions) of ``t``
    (``_get_expr_variables``, ``independence_solver.py:10-22``)."""
    return sorted({n for _, n in _symbols(t)})


def _symbols(t: T.Term):
    out = set()
    for n in T.postorder([t]):
        if n.op in ("bvvar", "boolvar", "array_var"):
            out.add(("v", n.params[0]))
        elif n.op == "app":
            name = n.params[0]
            out.add(("f", name[:-2] if name.endswith("-1") else name))
    return out


class DependenceBucket:
    """Conditions that depend on each other, and their variables (``independence_solver.py:25-35``)."""

    def __init__(self, variables=None, conditions=None):
        self.variables: set = set(variables or ())
        self.conditions: List[T.Term] = list(conditions or [])


class DependenceMap:
    """Union of constraints into variable-disjoint buckets (``independence_solver.py:38-82``).
    Variable-free conditions are kept in one bucket of their own (``ground``)."""

    def __init__(self):
        self.buckets: List[DependenceBucket] = []
        self.variable_map: Dict[tuple, DependenceBucket] = {}
        self.ground = DependenceBucket()
        self._pos: Dict[int, int] = {}

    def add_condition(self, c: T.Term) -> None:
        self._pos.setdefault(c.id, len(self._pos))
        syms = _symbols(c)
        if not syms:
            self.ground.conditions.append(c)
            return
        relevant = []
        for s in syms:
            b = self.variable_map.get(s)
            if b is not None and all(b is not r for r in relevant):
                relevant.append(b)
        new = DependenceBucket(syms, [c])
        if relevant:
            for b in relevant:
                self.buckets.remove(b)
                new.variables |= b.variables
                new.conditions = b.conditions + new.conditions
            new.conditions.sort(key=lambda x: self._pos[x.id])
        self.buckets.append(new)
        for s in new.variables:
            self.variable_map[s] = new

    def result(self) -> List[List[T.Term]]:
        out = [b.conditions for b in sorted(self.buckets, key=lambda b: self._pos[b.conditions[0].id])]
        if self.ground.conditions:
            out.insert(0, list(self.ground.conditions))
        return out


def partition(constraints: Sequence[T.Term]) -> List[List[T.Term]]:
    """Buckets of ``constraints`` that share no symbol, ordered by their first
    condition; conditions keep their input order inside a bucket."""
    dm = DependenceMap()
    for c in constraints:
        dm.add_condition(c)
    return dm.result()
