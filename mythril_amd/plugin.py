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
import time
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

    def __repr__(self):
        return (f"mythgpu: {self.queries} queries, {self.gpu_models} GPU models, {self.fallbacks} to z3 "
                f"({self.unsupported} unsupported, {self.errors} errors, {self.rejected} rejected), "
                f"{self.candidates} candidates in {self.gpu_time:.3f} s")


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


def _record(dt: float, gpu_model: bool) -> None:
    """Feed the hook's work into LASER's ``SolverStatistics`` (what ``--solver-log`` /
    the statistics report print): a query the GPU answered never reaches the
    ``stat_smt_query``-wrapped z3 check, so it is counted here, with its time; the GPU
    counters ride along as extra attributes of the same singleton."""
    st = _solver_statistics()
    if st is None:
        return
    if gpu_model and getattr(st, "enabled", False):
        st.query_count += 1
        st.solver_time += dt
    st.gpu_models = STATS.gpu_models
    st.gpu_candidates = STATS.candidates
    st.gpu_time = STATS.gpu_time


def gpu_first(original):
    """Build the cached hook around the reference's ``get_model``."""

    @lru_cache(maxsize=2 ** 23)
    def get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True):
        STATS.queries += 1
        if minimize or maximize or os.environ.get("MYTHGPU_DISABLE") == "1":
            return original(constraints, minimize, maximize, enforce_execution_time)
        model = None
        t0 = time.perf_counter()
        try:
            model = _try_gpu(constraints, enforce_execution_time)
        except Exception as e:  # never raise a new exception type into LASER
            from .ssa import Unsupported

            if isinstance(e, Unsupported):
                STATS.unsupported += 1
            else:
                STATS.errors += 1
                log.debug("mythgpu: engine error, falling back to z3: %s", e)
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
    return get_model


def _try_gpu(constraints, enforce_execution_time):
    """One GPU attempt at ``get_model`` (``support/model.py:15-49``): the budget is the
    smaller of the query's z3 budget (``args.solver_timeout``, minus the execution-time
    reserve the reference keeps) and the hook's slice ``MYTHGPU_BUDGET_MS``; the search
    escalates to the compiled kernel inside it (``search.search``, async compile).  A hit
    is re-checked by z3 (``pin_model``) with what is left of the query's z3 budget."""
    from mythril.laser.ethereum.time_handler import time_handler  # type: ignore
    from mythril.laser.smt import Model  # type: ignore
    from mythril.support.support_args import args  # type: ignore

    from . import z3bridge
    from .native import Engine
    from .search import search_partitioned

    t0 = time.perf_counter()
    if any(type(c) == bool and not c for c in constraints):
        return None  # the original raises UnsatError for this
    cs = [c for c in constraints if type(c) != bool]
    if not cs:
        return None
    total = float(args.solver_timeout)
    if enforce_execution_time:
        total = min(total, time_handler.time_remaining() - 500)
    budget = min(total, float(os.environ.get("MYTHGPU_BUDGET_MS", "200")))
    if budget <= 0:
        return None
    terms = z3bridge.to_terms(cs)
    res = search_partitioned(Engine.get(), terms, timeout_s=budget / 1000.0, max_candidates=1 << 40)
    STATS.candidates += res.scanned
    if res.index is None:
        return None
    ver, scalars, arrays, funcs, _ = res.model
    if not ver:
        return None
    from .solver import Model as GpuModel

    left_ms = total - (time.perf_counter() - t0) * 1e3
    if left_ms <= 0:
        return None
    z3m = z3bridge.pin_model(cs, GpuModel(scalars, arrays, funcs), timeout_ms=left_ms)
    if z3m is None:
        STATS.rejected += 1
        log.warning("mythgpu: z3 did not confirm a GPU model (kept on z3)")
        return None
    return Model([z3m])


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
