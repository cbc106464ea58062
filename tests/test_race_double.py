"""The z3 race in the ``get_model`` hook (``plugin._race``), on CPU against the z3py double.

The reference spends one z3 budget per query (``mythril/support/model.py:25-49``).  The hook
runs that same check (``Optimize``, same timeout) in a fresh context on a worker thread while
the GPU searches, and returns the first answer.  Pinned here:

* an UNSAT query costs z3's own time plus the hand-off (≤ 2 ms), not the GPU slice;
* a repeated UNSAT tuple is answered by the reference's z3 path without a GPU search;
* a GPU hit interrupts z3; a z3 ``sat`` cancels the GPU search; a model z3 does not confirm
  leaves z3's answer in charge;
* anything the GPU side cannot take (unsupported operator, no time left) goes to the
  reference's path unchanged; LASER's ``SolverStatistics`` counts every raced query.
"""
import statistics
import time

import pytest

from mythril_amd import plugin, z3bridge
from mythril_amd.search import SearchResult
from mythril_amd.ssa import Unsupported
from test_z3bridge_double import _hit, _query, _Stats, _UnsatError, fz3, mythril_standin, z3  # noqa: F401


def _wait_for(pred, timeout=2.0):
    t_end = time.perf_counter() + timeout
    while time.perf_counter() < t_end:
        if pred():
            return True
        time.sleep(0.001)
    return pred()


def test_race_unsat_costs_only_z3_time(mythril_standin):
    S = mythril_standin
    z3.Optimize.DELAY, z3.Optimize.ANSWER = 0.03, z3.unsat
    S.state.result, S.state.delay = SearchResult(None, 0, 1 << 30, 0.2), 0.2  # the GPU would search 200 ms
    hooked = plugin.gpu_first(S.original)
    over = []
    for _ in range(7):
        cs = tuple(_query())
        t0 = time.perf_counter()
        with pytest.raises(_UnsatError):
            hooked(cs)
        dt = time.perf_counter() - t0
        over.append(dt - z3.Optimize.calls[-1][2])
        assert _wait_for(lambda: len(S.state.cancelled) == len(over))  # the GPU search was stopped
    # what a miss adds to z3's own time: the hand-off, not the GPU's 200-ms slice (a few ms at most on a
    # loaded host: 2-5 ms measured with the suite running 8 ways)
    assert statistics.median(over) <= 10e-3, over
    assert not S.calls  # the reference's path never ran: z3 answered once, in the race
    # the race ran the reference's check: its timeout, on a worker thread
    name, timeout, _, result = z3.Optimize.calls[-1]
    # min(solver_timeout, remaining - 500), less the time the check waited for a z3 worker (a few
    # ms when the machine is loaded)
    assert name.startswith("mythgpu-z3") and 9_300 <= timeout <= 9_500 and result is z3.unsat
    assert plugin.STATS.z3_answers == 7 and plugin.STATS.races == 7
    assert _Stats().query_count == 7  # counted where stat_smt_query would have counted it


def test_race_repeated_unsat_skips_the_gpu(mythril_standin):
    S = mythril_standin
    z3.Optimize.ANSWER = z3.unsat
    S.state.result = SearchResult(None, 0, 1 << 20, 0.001)
    hooked = plugin.gpu_first(S.original)
    cs = tuple(_query())
    with pytest.raises(_UnsatError):
        hooked(cs)
    searches = len(S.state.budgets)
    assert hooked(cs) == "z3-model"  # the reference's get_model, unchanged
    assert len(S.state.budgets) == searches and S.calls == [cs]
    assert plugin.STATS.negative_hits == 1
    # a bounded LRU
    neg = plugin.NegativeCache(size=2)
    for k in range(3):
        neg.add((k,))
    assert (0,) not in neg and (1,) in neg and (2,) in neg and len(neg) == 2
    neg.add([1])  # unhashable: ignored
    assert [1] not in neg


def test_race_gpu_hit_interrupts_z3(mythril_standin):
    S = mythril_standin
    z3.Optimize.DELAY, z3.Optimize.ANSWER = 5.0, z3.sat
    S.state.result = _hit()
    hooked = plugin.gpu_first(S.original)
    t0 = time.perf_counter()
    m = hooked(tuple(_query()))
    assert time.perf_counter() - t0 < 1.0
    assert m.raw[0].ctx is z3.main_ctx() and m.raw[0].env[0]["x"] == 5  # the GPU model, pinned by z3
    assert _wait_for(lambda: z3.Optimize.calls and z3.Optimize.calls[-1][3] is z3.unknown)  # interrupted
    assert plugin.STATS.gpu_models == 1 and _Stats().query_count == 1


def test_race_z3_sat_first_cancels_gpu(mythril_standin):
    S = mythril_standin
    z3.Optimize.DELAY, z3.Optimize.ANSWER = 0.005, z3.sat
    S.state.result, S.state.delay = _hit(), 0.5
    hooked = plugin.gpu_first(S.original)
    t0 = time.perf_counter()
    m = hooked(tuple(_query()))
    assert time.perf_counter() - t0 < 0.2
    assert m.raw[0].ctx is z3.main_ctx() and m.raw[0].env == ({}, {}, {})  # z3's own model
    assert _wait_for(lambda: S.state.cancelled)
    assert plugin.STATS.gpu_models == 0 and plugin.STATS.z3_answers == 1


def test_race_rejected_gpu_model_waits_for_z3(mythril_standin):
    S = mythril_standin
    z3.Optimize.DELAY, z3.Optimize.ANSWER = 0.02, z3.unknown  # z3 ran out of time
    S.state.result = _hit(ok=False)
    hooked = plugin.gpu_first(S.original)
    with pytest.raises(_UnsatError):
        hooked(tuple(_query()))
    assert plugin.STATS.rejected == 1 and plugin.STATS.gpu_models == 0 and not S.calls


def test_race_engine_error_leaves_z3_answer(mythril_standin):
    S = mythril_standin
    z3.Optimize.DELAY, z3.Optimize.ANSWER = 0.05, z3.sat  # the GPU side fails first
    S.state.raise_ = RuntimeError("engine")
    m = plugin.gpu_first(S.original)(tuple(_query()))
    assert m.raw[0].env == ({}, {}, {}) and plugin.STATS.errors == 1


def test_race_reference_path_when_nothing_to_race(mythril_standin, monkeypatch):
    S = mythril_standin
    hooked = plugin.gpu_first(S.original)
    # no execution time left / literal False: the reference raises UnsatError itself
    S.th.remaining = 100.0
    assert hooked(tuple(_query())) == "z3-model"
    S.th.remaining = 10_000.0
    assert hooked((False,) + tuple(_query())) == "z3-model"
    # an operator the engine does not run
    monkeypatch.setattr(z3bridge, "to_terms", lambda cs: (_ for _ in ()).throw(Unsupported("op")))
    assert hooked(tuple(_query())) == "z3-model"
    assert plugin.STATS.unsupported == 1 and len(S.calls) == 3 and not z3.Optimize.calls
    assert not S.state.budgets  # the GPU never searched


def test_race_solver_time_is_z3_check_time(mythril_standin):
    """``SolverStatistics.solver_time`` gets z3's own check seconds for a z3-answered race (what
    ``stat_smt_query`` times, ``solver_statistics.py:16-22``), not the hook's wall time."""
    S = mythril_standin
    z3.Optimize.DELAY, z3.Optimize.ANSWER = 0.03, z3.unsat
    S.state.result, S.state.delay = SearchResult(None, 0, 1 << 20, 0.01), 0.01
    hooked = plugin.gpu_first(S.original)
    before = _Stats().solver_time
    with pytest.raises(_UnsatError):
        hooked(tuple(_query()))
    check_s = z3.Optimize.calls[-1][2]
    assert _Stats().solver_time - before == pytest.approx(check_s, abs=2e-4)


def test_race_lingering_interrupted_checks(mythril_standin):
    """Two checks the GPU beat keep running after ``Z3_interrupt`` (LINGER): the next query's z3
    check waits for a worker, its timeout is what is left of the query budget, and an
    ``unknown`` it returns beside an interrupted check is counted."""
    S = mythril_standin
    z3.Optimize.DELAY, z3.Optimize.ANSWER, z3.Optimize.LINGER = 5.0, z3.sat, 0.15
    S.state.result = _hit()
    hooked = plugin.gpu_first(S.original)
    for k in range(2):
        hooked(tuple(_query()))  # GPU wins twice; both z3 checks linger 150 ms
    assert plugin.STATS.gpu_models == 2
    z3.Optimize.DELAY, z3.Optimize.ANSWER, z3.Optimize.LINGER = 0.01, z3.unknown, 0.0
    S.state.result = SearchResult(None, 0, 1 << 20, 0.001)
    cs = tuple(_query())
    with pytest.raises(_UnsatError):
        hooked(cs)
    assert _wait_for(lambda: len(z3.Optimize.calls) == 3)
    timeout = min(c[1] for c in z3.Optimize.calls)
    assert timeout <= 9_500 - 100  # queued ~150 ms behind the lingering pair
    assert plugin.STATS.z3_queued_ms >= 100
    # the first lingering check ended as this one started, the second was still running
    assert plugin.STATS.z3_unknown_beside_interrupted == 1
    assert cs not in plugin.NEGATIVE  # an unknown on a cut budget is not cached


def test_race_confirm_error_waits_for_z3(mythril_standin, monkeypatch):
    """A z3 error while re-checking a GPU hit is counted and z3's own answer is returned."""
    S = mythril_standin
    z3.Optimize.DELAY, z3.Optimize.ANSWER = 0.02, z3.sat
    S.state.result = _hit()
    monkeypatch.setattr(z3bridge, "pin_model", lambda *a, **k: (_ for _ in ()).throw(RuntimeError("z3")))
    m = plugin.gpu_first(S.original)(tuple(_query()))
    assert m.raw[0].env == ({}, {}, {}) and plugin.STATS.errors == 1 and plugin.STATS.gpu_models == 0
