"""Solver-side mirror of the reference's hot path, answered by the GPU engine.

Same names and contracts as the reference:

* ``get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True)``
  — ``mythril/support/model.py:15-49``: ``lru_cache``d; a literal ``False``
  constraint, an exhausted time budget, unsat or unknown all raise
  :class:`UnsatError`; Python ``bool`` constraints are filtered out.
* ``Solver`` / ``Optimize`` with ``add/append/set_timeout/check/model``
  (``mythril/laser/smt/solver/solver.py:15-105``), ``check`` wrapped by
  ``stat_smt_query`` into ``SolverStatistics`` (``solver_statistics.py:8-43``).
* ``Model`` with ``decls/__getitem__/eval(expr, model_completion)``
  (``mythril/laser/smt/model.py:6-59``).

Differences, by construction of the engine: ``check`` returns ``sat`` (a model
found by the GPU search) or ``unknown`` — never ``unsat``; objectives
(``minimize``/``maximize``) are not optimised here (inside Mythril those queries
stay on z3, see ``plugin.py``); ``Model.eval`` evaluates on the GPU.
"""
from __future__ import annotations

import logging
import time
from functools import lru_cache
from typing import Dict, List, Optional, Sequence, Tuple

from . import search, ssa
from .smt import Bool, Expression
from .smt import terms as T

log = logging.getLogger("mythgpu")

try:  # the reference's own exception type when Mythril is importable
    from mythril.exceptions import UnsatError  # type: ignore
except Exception:  # pragma: no cover - Mythril absent in this image

    class UnsatError(Exception):
        """Mirror of ``mythril.exceptions.UnsatError`` (``exceptions.py:16-20``)."""


class CheckSatResult:
    def __init__(self, name: str):
        self.name = name

    def __repr__(self):
        return self.name

    def __eq__(self, other):
        return isinstance(other, CheckSatResult) and other.name == self.name

    def __hash__(self):
        return hash(self.name)


sat = CheckSatResult("sat")
unsat = CheckSatResult("unsat")
unknown = CheckSatResult("unknown")


class _Singleton(type):
    _instances: Dict[type, object] = {}

    def __call__(cls, *a, **k):
        if cls not in cls._instances:
            cls._instances[cls] = super().__call__(*a, **k)
        return cls._instances[cls]


class Args(metaclass=_Singleton):
    """``mythril/support/support_args.py:1-16`` (only what the hot path reads)."""

    def __init__(self):
        self.solver_timeout = 10000
        self.sparse_pruning = True


args = Args()


class TimeHandler(metaclass=_Singleton):
    """``mythril/laser/ethereum/time_handler.py:5-18``."""

    def __init__(self):
        self._start_time = int(time.time() * 1000)
        self._execution_time = 86400 * 1000

    def start_execution(self, execution_time):
        self._start_time = int(time.time() * 1000)
        self._execution_time = execution_time * 1000

    def time_remaining(self):
        return self._execution_time - (int(time.time() * 1000) - self._start_time)


time_handler = TimeHandler()


class SolverStatistics(metaclass=_Singleton):
    """``solver_statistics.py:28-43`` plus the engine's own counters."""

    def __init__(self):
        self.enabled = False
        self.query_count = 0
        self.solver_time = 0.0
        self.gpu_sat = 0
        self.gpu_unknown = 0
        self.candidates = 0

    def __repr__(self):
        return (f"Query count: {self.query_count} \nSolver time: {self.solver_time}\n"
                f"GPU sat: {self.gpu_sat}, GPU unknown: {self.gpu_unknown}, candidates: {self.candidates}")


def stat_smt_query(func):
    stat_store = SolverStatistics()

    def wrapper(*a, **k):
        if not stat_store.enabled:
            return func(*a, **k)
        stat_store.query_count += 1
        t0 = time.time()
        r = func(*a, **k)
        stat_store.solver_time += time.time() - t0
        return r

    return wrapper


def _raw(x) -> T.Term:
    return x.raw if isinstance(x, Expression) else x


class Value:
    """A concrete value returned by :meth:`Model.eval` (z3 ``BitVecNumRef``-like)."""

    __slots__ = ("v", "width", "is_bool")

    def __init__(self, v: int, width: int, is_bool: bool):
        self.v, self.width, self.is_bool = v, width, is_bool

    def as_long(self) -> int:
        return self.v

    def size(self) -> int:
        return self.width

    def __eq__(self, other):
        if isinstance(other, Value):
            return self.v == other.v
        return self.v == other

    def __hash__(self):
        return hash(self.v)

    def __repr__(self):
        return ("True" if self.v else "False") if self.is_bool else str(self.v)


class Model:
    """A finite model: scalar values plus array/UF tables with an ``else`` of 0."""

    def __init__(self, scalars=None, arrays=None, funcs=None):
        self.scalars: Dict[str, int] = dict(scalars or {})
        self.arrays: Dict[str, Tuple[Dict[int, int], int]] = dict(arrays or {})
        self.funcs: Dict[str, Tuple[Dict[int, int], int]] = dict(funcs or {})

    def decls(self) -> List[str]:
        return list(self.scalars) + list(self.arrays) + list(self.funcs)

    def __getitem__(self, item):
        name = item if isinstance(item, str) else _raw(item).params[0]
        if name in self.scalars:
            return self.scalars[name]
        if name in self.arrays:
            return self.arrays[name]
        if name in self.funcs:
            return self.funcs[name]
        return None

    def substitute(self, t: T.Term, model_completion: bool = True) -> T.Term:
        """Replace every symbol by its interpretation (arrays -> stores over K(else),
        functions -> ite chains over their table)."""
        memo: Dict[int, T.Term] = {}
        for n in T.postorder([t]):
            args = tuple(memo[a.id] for a in n.args)
            op = n.op
            if op in ("bvvar", "boolvar"):
                name = n.params[0]
                if name in self.scalars or model_completion:
                    v = self.scalars.get(name, 0)
                    r = T.BoolVal(bool(v)) if op == "boolvar" else T.BitVecVal(v, n.width)
                else:
                    r = n
            elif op == "array_var":
                table, dflt = self.arrays.get(n.params[0], ({}, 0))
                _, d, rng = n.sort
                r = T.ConstArray(d, T.BitVecVal(dflt, rng))
                for k, v in table.items():
                    r = T.store(r, T.BitVecVal(k, d), T.BitVecVal(v, rng))
            elif op == "app":
                fname, dom, rng = n.params
                table, dflt = self.funcs.get(fname, ({}, 0))
                r = T.BitVecVal(dflt, rng)
                for k, v in table.items():
                    r = T.ite(T.eq(args[0], T.BitVecVal(k, dom)), T.BitVecVal(v, rng), r)
            else:
                r = n if args == n.args else T.mk(n.op, n.sort, args, n.params)
            memo[n.id] = r
        return memo[t.id]

    def eval_many(self, expressions, model_completion: bool = True) -> List["Value"]:
        """Batched :meth:`eval`: every ground term is watched in ONE program and
        evaluated by one ``mg_eval`` launch (terms with unbound symbols come back
        symbolic, as in :meth:`eval`)."""
        from .native import Engine

        subs = [self.substitute(_raw(e), model_completion) for e in expressions]
        ground = [t for t in subs if not T.free_symbols([t])]
        out: Dict[int, Value] = {}
        if ground:
            P = ssa.flatten([T.BoolVal(True)], extra=ground)
            P.set_watch([P.term_node[t.id] for t in ground])
            eng = Engine.get()
            prog = eng.load(P.to_bytes())
            try:
                info = eng.info(prog)
                _, watch = eng.eval(prog, ssa.soa_from_assignments(P, [[]]), 1, watch_words=info.watch_words)
            finally:
                eng.free(prog)
            r = 0
            for t in ground:
                L = ssa.limbs(t.width)
                out[t.id] = Value(ssa.limbs_to_int(watch[r:r + L, 0]), t.width, t.is_bool)
                r += L
        return [out.get(t.id, t) for t in subs]

    def eval(self, expression, model_completion: bool = False):
        """Evaluate on the GPU (``mg_eval`` of the ground, substituted term)."""
        from .native import Engine

        t = self.substitute(_raw(expression), model_completion)
        if T.free_symbols([t]):
            return t  # symbols without interpretation stay symbolic (as z3 does)
        P = ssa.flatten([T.BoolVal(True)], extra=[t])
        P.set_watch([P.term_node[t.id]])
        eng = Engine.get()
        prog = eng.load(P.to_bytes())
        try:
            info = eng.info(prog)
            _, watch = eng.eval(prog, ssa.soa_from_assignments(P, [[]]), 1, watch_words=info.watch_words)
        finally:
            eng.free(prog)
        v = ssa.limbs_to_int(watch[:, 0])
        return Value(v, t.width, t.is_bool)


def _solve(constraints: Sequence[T.Term], timeout_ms: float) -> Optional[Model]:
    """GPU search for a model of the conjunction within the time budget."""
    from .native import Engine

    st = SolverStatistics()
    eng = Engine.get()
    res = search.search_partitioned(eng, list(constraints), timeout_s=max(timeout_ms, 1.0) / 1000.0,
                                    max_candidates=1 << 40)
    st.candidates += res.scanned
    if res.index is None:
        st.gpu_unknown += 1
        return None
    ver, scalars, arrays, funcs, _ = res.model
    if not ver:
        st.gpu_unknown += 1
        return None
    st.gpu_sat += 1
    return Model(scalars, arrays, funcs)


class BaseSolver:
    def __init__(self):
        self.constraints: List[T.Term] = []
        self.timeout = args.solver_timeout
        self._model: Optional[Model] = None

    def set_timeout(self, timeout: int) -> None:
        self.timeout = timeout

    def add(self, *constraints) -> None:
        for c in constraints:
            if isinstance(c, (list, tuple)):
                self.add(*c)
            else:
                self.constraints.append(_raw(c) if not isinstance(c, bool) else T.BoolVal(c))

    def append(self, *constraints) -> None:
        self.add(*constraints)

    @stat_smt_query
    def check(self, *assumptions) -> CheckSatResult:
        cs = self.constraints + [_raw(a) for a in assumptions]
        if any(c.op == "boolconst" and not c.params[0] for c in cs):
            self._model = None
            return unknown
        cs = [c for c in cs if c.op != "boolconst"]
        self._model = _solve(cs, self.timeout) if cs else Model()
        return sat if self._model is not None else unknown

    def model(self) -> Model:
        if self._model is None:
            raise UnsatError("no model (last check was not sat)")
        return self._model


class Solver(BaseSolver):
    def reset(self) -> None:
        self.constraints = []
        self._model = None

    def pop(self, num: int) -> None:
        self.constraints = self.constraints[: max(0, len(self.constraints) - num)]


class IndependenceSolver(Solver):
    """``mythril/laser/smt/solver/independence_solver.py:85-153``: every
    :class:`BaseSolver` here already splits its constraints into
    variable-disjoint buckets before the GPU search (``search_partitioned``)
    and returns the merged model, so this is the same solver under the
    reference's name."""


class Optimize(BaseSolver):
    def __init__(self):
        super().__init__()
        self.objectives: List[Tuple[str, T.Term]] = []

    def minimize(self, element) -> None:
        self.objectives.append(("min", _raw(element)))

    def maximize(self, element) -> None:
        self.objectives.append(("max", _raw(element)))


@lru_cache(maxsize=2 ** 23)
def get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True):
    """``mythril/support/model.py:15-49`` over the GPU engine."""
    s = Optimize()
    timeout = args.solver_timeout
    if enforce_execution_time:
        timeout = min(timeout, time_handler.time_remaining() - 500)
        if timeout <= 0:
            raise UnsatError
    s.set_timeout(timeout)
    for constraint in constraints:
        if type(constraint) == bool and not constraint:
            raise UnsatError
    constraints = [constraint for constraint in constraints if type(constraint) != bool]
    for constraint in constraints:
        s.add(constraint)
    for e in minimize:
        s.minimize(e)
    for e in maximize:
        s.maximize(e)
    result = s.check()
    if result == sat:
        return s.model()
    elif result == unknown:
        log.debug("GPU search exhausted its budget without a model")
    raise UnsatError
