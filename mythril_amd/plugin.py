"""LaserPlugin + pre-solve hook: the drop-in boundary inside Mythril.

How it gets control (reference call path):
``cli.py:38`` -> ``MythrilPluginLoader`` -> entry point group ``mythril.plugins``
(``plugin/discovery.py:17-21``) -> ``LaserPluginLoader.load`` -> ``SymExecWrapper``
-> ``instrument_virtual_machine`` -> ``builder(**args).initialize(laser)``
(``laser/plugin/loader.py:53-72``).  ``initialize`` installs the hook.

The hook wraps ``mythril.support.model.get_model`` (``support/model.py:15-49``)
at the names its callers bound at import time
(``laser/ethereum/state/constraints.py:5``, ``analysis/solver.py:6``):

* queries with objectives (``minimize``/``maximize`` — the model values are
  printed in reports, ``analysis/solver.py:48-96``) go to z3 unchanged;
* otherwise the constraint DAG is flattened (``z3bridge``) and the GPU searches
  for a model within a slice of the solver budget; a hit is re-checked by z3
  in a fresh solver (``z3bridge.pin_model``) and returned as the reference's own
  ``Model([z3.ModelRef])``; anything else — unsupported operator, no hit, any
  engine error — falls through to the original z3 path, so the hook can only
  return earlier with ``sat``, never change a verdict.

Control without CLI changes: ``MYTHGPU_DISABLE=1`` turns the hook off,
``MYTHGPU_BUDGET_MS`` caps the GPU slice (default 200 ms),
``MYTHGPU_DEVICE`` picks the GPU.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from collections import OrderedDict
from concurrent.futures import FIRST_COMPLETED, ThreadPoolExecutor, wait
from functools import lru_cache

log = logging.getLogger("mythgpu")

try:  # the reference's plugin API when Mythril is importable
    from mythril.laser.plugin.builder import PluginBuilder  # type: ignore
    from mythril.laser.plugin.interface import LaserPlugin  # type: ignore
    from mythril.plugin.interface import MythrilLaserPlugin  # type: ignore

    HAVE_MYTHRIL = True
except Exception:  # stand-ins with the reference's shape (builder.py:7-21, interface.py:4-23, 39-45)
    HAVE_MYTHRIL = False

    class LaserPlugin:  # type: ignore[no-redef]
        def initialize(self, symbolic_vm) -> None:
            raise NotImplementedError

    class PluginBuilder:  # type: ignore[no-redef]
        plugin_name = "Default Plugin Name"

        def __init__(self):
            self.enabled = True

        def __call__(self, *args, **kwargs) -> LaserPlugin:
            raise NotImplementedError

    class MythrilLaserPlugin(PluginBuilder):  # type: ignore[no-redef]
        author = "Default Author"
        name = "Plugin Name"
        plugin_license = "All rights reserved."
        plugin_type = "Mythril Plugin"
        plugin_version = "0.0.1 "
        plugin_description = "This is an example plugin description"


class HookStats:
    def __init__(self):
        self.queries = 0
        self.gpu_models = 0
        self.fallbacks = 0
        self.unsupported = 0
        self.errors = 0
        self.rejected = 0      # GPU models z3 did not confirm (kept on z3)
        self.candidates = 0    # candidate assignments the GPU evaluated
        self.gpu_time = 0.0    # seconds inside the GPU attempt (hits and misses)
        self.races = 0         # queries raced against z3
        self.z3_answers = 0    # raced queries z3 answered (GPU miss or slower)
        self.race_z3_time = 0.0   # z3 check seconds of those
        self.race_overhead = 0.0  # hook wall time beyond z3's own, summed over them
        self.negative_hits = 0    # repeats of a GPU-missed unsat/unknown tuple sent straight to z3
        self.z3_queued_ms = 0.0   # raced z3 checks' waits for a worker (interrupted checks lingering)
        self.z3_unknown_beside_interrupted = 0  # z3 unknowns while an interrupted check still ran

    def __repr__(self):
        return (f"mythgpu: {self.queries} queries, {self.gpu_models} GPU models, {self.fallbacks} to z3 "
                f"({self.unsupported} unsupported, {self.errors} errors, {self.rejected} rejected), "
                f"{self.candidates} candidates in {self.gpu_time:.3f} s; {self.races} raced, "
                f"{self.z3_answers} by z3 (+{self.race_overhead * 1e3:.1f} ms over z3), "
                f"{self.negative_hits} negative-cache repeats, {self.z3_unknown_beside_interrupted} z3 unknown "
                f"beside an interrupted check")


STATS = HookStats()
_ORIGINAL = None
_ORIGINAL_SHA = None


def _solver_statistics():
    """LASER's ``SolverStatistics`` singleton (``laser/smt/solver/solver_statistics.py:29-45``),
    or None without Mythril."""
    try:
        from mythril.laser.smt.solver.solver_statistics import SolverStatistics  # type: ignore
    except Exception:
        return None
    return SolverStatistics()


def _record(dt: float, answered: bool) -> None:
    """Feed the hook's work into LASER's ``SolverStatistics`` (what ``--solver-log`` /
    the statistics report print): a query the GPU answered never reaches the
    ``stat_smt_query``-wrapped z3 check, so it is counted here, with its time (the hook's
    wall time); a query z3 answered in the race is counted with z3's own check seconds, as
    ``stat_smt_query`` times only the check (``solver_statistics.py:16-22``).  The GPU
    counters ride along as extra attributes of the same singleton."""
    st = _solver_statistics()
    if st is None:
        return
    if answered and getattr(st, "enabled", False):
        st.query_count += 1
        st.solver_time += dt
    st.gpu_models = STATS.gpu_models
    st.gpu_candidates = STATS.candidates
    st.gpu_time = STATS.gpu_time


class NegativeCache:
    """Bounded LRU set of constraint tuples that the GPU missed AND z3 answered unsat/unknown.
    Keys are the tuples ``get_model`` receives, hashed and compared exactly as its
    ``lru_cache`` does (``Bool.__hash__``/``__eq__``, ``laser/smt/bool.py:50-84``).  A repeat
    goes straight to the reference's z3 path: the ``lru_cache`` does not cache ``UnsatError``,
    and LASER re-asks (``Constraints.is_possible`` per successor, ``svm.py:252-257``; the
    modules at the end of a transaction)."""

    def __init__(self, size: int = 4096):
        self.size = size
        self._d = OrderedDict()

    def __contains__(self, key) -> bool:
        try:
            if key in self._d:
                self._d.move_to_end(key)
                return True
        except Exception:  # an unhashable/uncomparable key is simply not cached
            pass
        return False

    def add(self, key) -> None:
        try:
            self._d[key] = True
            self._d.move_to_end(key)
        except Exception:
            return
        while len(self._d) > self.size:
            self._d.popitem(last=False)

    def clear(self) -> None:
        self._d.clear()

    def __len__(self) -> int:
        return len(self._d)


NEGATIVE = NegativeCache()
# z3 runs on its own worker threads, the GPU search on one more: ctypes releases the GIL inside
# ``Z3_optimize_check`` and inside every engine call, so both make progress while the calling
# thread waits for the first answer.  Two z3 workers: an interrupted check that is slow to
# notice ``Z3_interrupt`` does not hold up the next query's.
_Z3_POOL = ThreadPoolExecutor(max_workers=2, thread_name_prefix="mythgpu-z3")
# z3 checks the GPU beat that are still running (``Z3_interrupt`` is noticed at z3's next
# checkpoint): a new check starts only on a free worker, so at most two of them compete with it
_LINGER = threading.Lock()
_LINGERING = [0]
_GPU_POOL = ThreadPoolExecutor(max_workers=1, thread_name_prefix="mythgpu-gpu")
# longest single launch while racing: after z3 answers, the engine is free within this
RACE_LAUNCH_S = 0.002


class Z3Race:
    """The reference's own check of the query (``support/model.py:25-49``: ``Optimize``, the
    same timeout, no objectives), run in a fresh ``z3.Context`` on a worker thread.  The
    constraints are translated on the calling thread (LASER's main context is not
    thread-safe); the worker touches only the fresh context.  ``interrupt`` is
    ``Z3_interrupt`` on that context, which z3 allows from any thread."""

    def __init__(self, z3, constraints, timeout_ms: int):
        self.z3 = z3
        self.ctx = z3.Context()
        self.raws = [getattr(c, "raw", c).translate(self.ctx) for c in constraints]
        self.timeout_ms = max(1, int(timeout_ms))
        self.result = None
        self.model = None
        self.seconds = 0.0        # z3's own check, from its real start (what stat_smt_query times)
        self.queued_ms = 0.0      # submission -> a free worker
        self.beside_interrupted = 0  # interrupted checks still running when this one started
        self.submitted = time.perf_counter()
        self._interrupted = False
        self._finished = False

    def run(self):
        z3 = self.z3
        t_start = time.perf_counter()
        self.queued_ms = (t_start - self.submitted) * 1e3
        with _LINGER:
            self.beside_interrupted = _LINGERING[0]
        try:
            s = z3.Optimize(ctx=self.ctx)
            # the budget left of the reference's timeout: a check that waited for a worker (two
            # interrupted checks still running) does not end past the query's wall-clock budget
            s.set("timeout", max(1, self.timeout_ms - int(self.queued_ms)))
            s.add(*self.raws)
            t0 = time.perf_counter()
            self.result = s.check()
            self.seconds = time.perf_counter() - t0
            if self.result == z3.sat:
                self.model = s.model()
        finally:
            with _LINGER:
                self._finished = True
                if self._interrupted:
                    _LINGERING[0] -= 1
        return self

    def interrupt(self) -> None:
        with _LINGER:
            if not self._finished and not self._interrupted:
                self._interrupted = True
                _LINGERING[0] += 1
        try:
            self.ctx.interrupt()
        except Exception:  # pragma: no cover - the check already ended
            pass


def race(gpu_job, z3_job, confirm):
    """First answer of two workers: ``gpu_job(cancel)`` on the GPU thread and ``z3_job.run()``
    on a z3 thread.  A GPU result that ``confirm`` turns into a model wins (``z3_job`` is then
    interrupted): ``("gpu", model)``.  Otherwise z3's answer is awaited: ``("z3", z3_job.run()'s
    value)``; a z3 exception propagates.  ``cancel`` is set on every exit, so a GPU search still
    running stops at its next launch boundary.  GPU-side exceptions are counted, never raised."""
    cancel = threading.Event()
    f_z3 = _Z3_POOL.submit(z3_job.run)
    f_gpu = _GPU_POOL.submit(gpu_job, cancel)
    try:
        done, _ = wait([f_z3, f_gpu], return_when=FIRST_COMPLETED)
        if f_z3 not in done:
            res = None
            try:
                res = f_gpu.result()
            except Exception as e:
                _count_error(e)
            model = None
            try:  # a z3 error re-checking the hit, or a model that does not decode: z3's answer stands
                model = confirm(res)
            except Exception as e:
                _count_error(e)
            if model is not None:
                z3_job.interrupt()
                return "gpu", model
        return "z3", f_z3.result()
    finally:
        cancel.set()


def _unsat_error():
    from mythril.exceptions import UnsatError  # type: ignore

    return UnsatError


def gpu_first(original):
    """Build the cached hook around the reference's ``get_model``.

    With ``MYTHGPU_RACE`` unset or ``1`` (the default) the GPU search and the reference's z3
    check race (``_race``): a GPU miss then costs only the hand-off, not the GPU slice.  With
    ``MYTHGPU_RACE=0`` the GPU searches first and z3 runs after a miss (``_try_gpu``)."""

    @lru_cache(maxsize=2 ** 23)
    def get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True):
        STATS.queries += 1
        if minimize or maximize or os.environ.get("MYTHGPU_DISABLE") == "1":
            return original(constraints, minimize, maximize, enforce_execution_time)
        if constraints in NEGATIVE:
            STATS.negative_hits += 1
            return original(constraints, minimize, maximize, enforce_execution_time)
        if os.environ.get("MYTHGPU_RACE", "1") != "0":
            return _race(original, constraints, enforce_execution_time)
        model = None
        t0 = time.perf_counter()
        try:
            model = _try_gpu(constraints, enforce_execution_time)
        except Exception as e:  # never raise a new exception type into LASER
            _count_error(e)
        dt = time.perf_counter() - t0
        STATS.gpu_time += dt
        if model is not None:
            STATS.gpu_models += 1
        _record(dt, model is not None)
        if model is not None:
            return model
        STATS.fallbacks += 1
        return original(constraints, minimize, maximize, enforce_execution_time)

    get_model.__wrapped_original__ = original
    get_model.negative_cache = NEGATIVE
    return get_model


def _count_error(e) -> None:
    from .ssa import Unsupported

    if isinstance(e, Unsupported):
        STATS.unsupported += 1
    else:
        STATS.errors += 1
        log.debug("mythgpu: engine error, falling back to z3: %s", e)


def _budgets(constraints, enforce_execution_time):
    """The reference's budget arithmetic (``support/model.py:26-31``): ``(cs, z3 budget ms,
    GPU slice ms)``, or None where the reference raises before solving (no time left, a
    literal ``False``) or where there is nothing to search (only literal ``True``)."""
    from mythril.laser.ethereum.time_handler import time_handler  # type: ignore
    from mythril.support.support_args import args  # type: ignore

    total = float(args.solver_timeout)
    if enforce_execution_time:
        total = min(total, time_handler.time_remaining() - 500)
    if total <= 0 or any(type(c) == bool and not c for c in constraints):
        return None
    cs = [c for c in constraints if type(c) != bool]
    if not cs:
        return None
    return cs, total, min(total, float(os.environ.get("MYTHGPU_BUDGET_MS", "200")))


def _race(original, constraints, enforce_execution_time):
    """z3 and the GPU on the same query, first answer wins (``get_model``'s contract,
    ``support/model.py:15-49``):

    * z3 answers first: the GPU search is cancelled (it stops at its next launch boundary,
      launches are at most ``RACE_LAUNCH_S`` long) and z3's answer is returned — ``sat`` as the
      reference's ``Model([z3.ModelRef])`` (translated back to the main context), ``unsat`` /
      ``unknown`` as ``UnsatError``, exactly as the reference raises;
    * the GPU hits first: the hit is re-checked by z3 (``pin_model``) and returned, and the z3
      worker is interrupted; a model z3 does not confirm is dropped and z3's answer awaited;
    * the GPU misses: z3's answer is awaited; a z3 ``unsat``/``unknown`` puts the tuple in the
      negative cache, so a repeat does not search again.

    Whatever the GPU side does — unsupported operator, engine error — only z3's answer can
    then come back, so the hook never changes a verdict and never raises a new exception
    type.  The hook's own z3 check is counted in LASER's ``SolverStatistics`` here, as
    ``stat_smt_query`` (``solver_statistics.py:8-25``) counts the reference's."""
    from . import z3bridge

    t0 = time.perf_counter()
    try:
        from mythril.laser.smt import Model  # type: ignore

        b = _budgets(constraints, enforce_execution_time)
    except Exception as e:  # no Mythril around the hook: nothing to race
        _count_error(e)
        b = None
    if b is None:
        return original(constraints, (), (), enforce_execution_time)
    cs, total, gpu_ms = b
    terms = None
    try:
        terms = z3bridge.to_terms(cs)
    except Exception as e:
        _count_error(e)
    if terms is None:  # nothing to race: the reference's path, unchanged
        STATS.fallbacks += 1
        return original(constraints, (), (), enforce_execution_time)
    z3 = z3bridge.z3
    try:
        zr = Z3Race(z3, cs, total)
    except Exception as e:  # translation refused: the reference's path, unchanged
        log.debug("mythgpu: cannot race z3 on this query: %s", e)
        STATS.fallbacks += 1
        return original(constraints, (), (), enforce_execution_time)
    STATS.races += 1
    winner, out = race(lambda cancel: _gpu_search(terms, gpu_ms / 1000.0, cancel), zr,
                       lambda res: _confirm(cs, res, total - (time.perf_counter() - t0) * 1e3))
    if winner == "gpu":
        STATS.gpu_models += 1
        _record(time.perf_counter() - t0, True)
        return Model([out])
    r = out
    STATS.z3_answers += 1
    dt = time.perf_counter() - t0
    STATS.race_z3_time += r.seconds
    STATS.race_overhead += max(0.0, dt - r.seconds)
    STATS.z3_queued_ms += r.queued_ms
    if r.result == z3.unknown and r.beside_interrupted:
        STATS.z3_unknown_beside_interrupted += 1
    _record(r.seconds, True)
    if r.result == z3.sat:
        return Model([r.model.translate(z3.main_ctx())])
    # the negative cache keeps unsat, and unknown only at the full solver timeout: a budget cut
    # by the execution timeout (or by a wait for a worker) may be what made z3 give up
    if r.result == z3.unsat or (r.queued_ms < 1.0 and total >= _full_timeout()):
        NEGATIVE.add(constraints)
    if r.result == z3.unknown:
        log.debug("Timeout encountered while solving expression using z3")
    raise _unsat_error()


def _full_timeout() -> float:
    try:
        from mythril.support.support_args import args  # type: ignore

        return float(args.solver_timeout)
    except Exception:
        return float("inf")


def _gpu_search(terms, budget_s, cancel):
    from .native import Engine
    from .search import search_partitioned

    t0 = time.perf_counter()
    try:
        res = search_partitioned(Engine.get(), terms, timeout_s=budget_s, max_candidates=1 << 40,
                                 cancel=cancel, max_launch_s=RACE_LAUNCH_S)
    finally:
        STATS.gpu_time += time.perf_counter() - t0
    STATS.candidates += res.scanned
    return res


def _confirm(cs, res, left_ms):
    """A GPU hit re-checked by z3 in a fresh context (``z3bridge.pin_model``), or None."""
    from . import z3bridge
    from .solver import Model as GpuModel

    if res is None or res.index is None or left_ms <= 0:
        return None
    ver, scalars, arrays, funcs, _ = res.model
    if not ver:
        return None
    z3m = z3bridge.pin_model(cs, GpuModel(scalars, arrays, funcs), timeout_ms=left_ms)
    if z3m is None:
        STATS.rejected += 1
        log.warning("mythgpu: z3 did not confirm a GPU model (kept on z3)")
    return z3m


def _try_gpu(constraints, enforce_execution_time):
    """One GPU attempt at ``get_model`` before z3 (``MYTHGPU_RACE=0``): the budget is the
    smaller of the query's z3 budget (``args.solver_timeout``, minus the execution-time
    reserve the reference keeps) and the hook's slice ``MYTHGPU_BUDGET_MS``; the search
    escalates to the compiled kernel inside it (``search.search``, async compile).  A hit
    is re-checked by z3 (``pin_model``) with what is left of the query's z3 budget."""
    from mythril.laser.smt import Model  # type: ignore

    from . import z3bridge
    from .native import Engine
    from .search import search_partitioned

    t0 = time.perf_counter()
    b = _budgets(constraints, enforce_execution_time)
    if b is None:
        return None
    cs, total, budget = b
    terms = z3bridge.to_terms(cs)
    res = search_partitioned(Engine.get(), terms, timeout_s=budget / 1000.0, max_candidates=1 << 40)
    STATS.candidates += res.scanned
    z3m = _confirm(cs, res, total - (time.perf_counter() - t0) * 1e3)
    return None if z3m is None else Model([z3m])


def batched_replace_with_actual_sha(concrete_transactions, model, code=None):
    """Drop-in for ``mythril.analysis.solver._replace_with_actual_sha`` (``analysis/solver.py:119-152``):
    the same scan and in-place replacements, with every preimage's Keccak-256 computed in one
    ``mg_keccak256`` launch instead of one ``sha3`` call per slice (``keccak_model.replace_with_actual_sha``)."""
    from mythril.laser.ethereum.keccak_function_manager import keccak_function_manager  # type: ignore
    from mythril.laser.smt import symbol_factory  # type: ignore

    from .keccak_model import replace_with_actual_sha
    from .native import Engine

    class _Manager:
        """LASER's manager, with the hashing moved to the GPU."""

        store_function = keccak_function_manager.store_function

        @staticmethod
        def get_concrete_hash_data(m, evaluate=None):
            return keccak_function_manager.get_concrete_hash_data(m)

        @staticmethod
        def find_concrete_keccaks(datas):
            digests = Engine.get().keccak256([d.value.to_bytes(d.size() // 8, "big") for d in datas])
            return [symbol_factory.BitVecVal(int.from_bytes(h, "big"), 256) for h in digests]

        @classmethod
        def find_concrete_keccak(cls, data):
            return cls.find_concrete_keccaks([data])[0]

    replace_with_actual_sha(concrete_transactions, model, _Manager, code=code,
                            evaluate=lambda terms: [model.eval(t) for t in terms], bvv=symbol_factory.BitVecVal)


def install() -> bool:
    """Patch the names ``get_model`` is bound to.  Idempotent; False without Mythril."""
    global _ORIGINAL
    if not HAVE_MYTHRIL:
        return False
    import mythril.analysis.solver as an_solver  # type: ignore
    import mythril.laser.ethereum.state.constraints as constraints_mod  # type: ignore
    import mythril.support.model as model_mod  # type: ignore

    global _ORIGINAL_SHA
    if _ORIGINAL is not None:
        return True
    _ORIGINAL = model_mod.get_model
    hooked = gpu_first(_ORIGINAL)
    model_mod.get_model = hooked
    constraints_mod.get_model = hooked
    an_solver.get_model = hooked
    # the transaction printer's Keccak fix-up (analysis/solver.py:88-92 calls it by module name)
    _ORIGINAL_SHA = getattr(an_solver, "_replace_with_actual_sha", None)
    if _ORIGINAL_SHA is not None:
        an_solver._replace_with_actual_sha = batched_replace_with_actual_sha
    return True


def uninstall() -> None:
    global _ORIGINAL, _ORIGINAL_SHA
    if _ORIGINAL is None or not HAVE_MYTHRIL:
        return
    import mythril.analysis.solver as an_solver  # type: ignore
    import mythril.laser.ethereum.state.constraints as constraints_mod  # type: ignore
    import mythril.support.model as model_mod  # type: ignore

    model_mod.get_model = constraints_mod.get_model = an_solver.get_model = _ORIGINAL
    if _ORIGINAL_SHA is not None:
        an_solver._replace_with_actual_sha = _ORIGINAL_SHA
    _ORIGINAL = _ORIGINAL_SHA = None


class MythgpuPlugin(LaserPlugin):
    """Installs the pre-solve hook and logs engine statistics at the end of the run
    (``svm.py:573-590`` ``laser_hook("stop_sym_exec")``)."""

    def initialize(self, symbolic_vm) -> None:
        installed = install()
        log.info("mythgpu: pre-solve hook %s", "installed" if installed else "unavailable")
        if hasattr(symbolic_vm, "laser_hook"):
            @symbolic_vm.laser_hook("stop_sym_exec")
            def _report():
                log.info("%r", STATS)


class MythgpuPluginBuilder(MythrilLaserPlugin):
    """Mythril plugin entry point (group ``mythril.plugins``, ``plugin/discovery.py:17-21``).

    ``MythrilPlugin.__init__`` does not chain to ``PluginBuilder.__init__``
    (``plugin/interface.py:22-23`` vs ``laser/plugin/builder.py:15-16``), so
    ``enabled`` is set here explicitly (read at ``laser/plugin/loader.py:61-64``)."""

    name = "mythgpu"
    plugin_name = "mythgpu"
    author = "mythril_amd"
    plugin_license = "MIT"
    plugin_type = "Laser Plugin"
    plugin_version = "0.1.0"
    plugin_description = "MI355X batched bit-vector search in front of z3 for get_model"
    plugin_default_enabled = True

    def __init__(self, *args, **kwargs):
        try:
            super().__init__(*args, **kwargs)
        except TypeError:
            super().__init__()
        self.enabled = True

    def __call__(self, *args, **kwargs):
        return MythgpuPlugin()
