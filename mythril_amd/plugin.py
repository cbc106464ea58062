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

    def __repr__(self):
        return (f"mythgpu: {self.queries} queries, {self.gpu_models} GPU models, {self.fallbacks} to z3 "
                f"({self.unsupported} unsupported, {self.errors} errors)")


STATS = HookStats()
_ORIGINAL = None


def gpu_first(original):
    """Build the cached hook around the reference's ``get_model``."""

    @lru_cache(maxsize=2 ** 23)
    def get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True):
        STATS.queries += 1
        if minimize or maximize or os.environ.get("MYTHGPU_DISABLE") == "1":
            return original(constraints, minimize, maximize, enforce_execution_time)
        model = None
        try:
            model = _try_gpu(constraints, enforce_execution_time)
        except Exception as e:  # never raise a new exception type into LASER
            from .ssa import Unsupported

            if isinstance(e, Unsupported):
                STATS.unsupported += 1
            else:
                STATS.errors += 1
                log.debug("mythgpu: engine error, falling back to z3: %s", e)
        if model is not None:
            STATS.gpu_models += 1
            return model
        STATS.fallbacks += 1
        return original(constraints, minimize, maximize, enforce_execution_time)

    get_model.__wrapped_original__ = original
    return get_model


def _try_gpu(constraints, enforce_execution_time):
    from mythril.laser.ethereum.time_handler import time_handler  # type: ignore
    from mythril.laser.smt import Model  # type: ignore
    from mythril.support.support_args import args  # type: ignore

    from . import z3bridge
    from .native import Engine
    from .search import search_partitioned

    if any(type(c) == bool and not c for c in constraints):
        return None  # the original raises UnsatError for this
    cs = [c for c in constraints if type(c) != bool]
    if not cs:
        return None
    budget = min(args.solver_timeout, float(os.environ.get("MYTHGPU_BUDGET_MS", "200")))
    if enforce_execution_time:
        budget = min(budget, time_handler.time_remaining() - 500)
    if budget <= 0:
        return None
    terms = z3bridge.to_terms(cs)
    res = search_partitioned(Engine.get(), terms, timeout_s=budget / 1000.0, max_candidates=1 << 34)
    if res.index is None:
        return None
    ver, scalars, arrays, funcs, _ = res.model
    if not ver:
        return None
    from .solver import Model as GpuModel

    z3m = z3bridge.pin_model(cs, GpuModel(scalars, arrays, funcs))
    if z3m is None:
        log.warning("mythgpu: z3 rejected a GPU model (kept on z3)")
        return None
    return Model([z3m])


def install() -> bool:
    """Patch the names ``get_model`` is bound to.  Idempotent; False without Mythril."""
    global _ORIGINAL
    if not HAVE_MYTHRIL:
        return False
    import mythril.analysis.solver as an_solver  # type: ignore
    import mythril.laser.ethereum.state.constraints as constraints_mod  # type: ignore
    import mythril.support.model as model_mod  # type: ignore

    if _ORIGINAL is not None:
        return True
    _ORIGINAL = model_mod.get_model
    hooked = gpu_first(_ORIGINAL)
    model_mod.get_model = hooked
    constraints_mod.get_model = hooked
    an_solver.get_model = hooked
    return True


def uninstall() -> None:
    global _ORIGINAL
    if _ORIGINAL is None or not HAVE_MYTHRIL:
        return
    import mythril.analysis.solver as an_solver  # type: ignore
    import mythril.laser.ethereum.state.constraints as constraints_mod  # type: ignore
    import mythril.support.model as model_mod  # type: ignore

    model_mod.get_model = constraints_mod.get_model = an_solver.get_model = _ORIGINAL
    _ORIGINAL = None


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
