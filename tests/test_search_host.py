"""Host logic of ``search.search`` (interpreter -> first tier -> O3 kernel) against a stand-in
engine: no GPU, no native library.

The stand-in answers every launch with "no hit" after a short sleep, so the search runs to its
budget; its compile tickets are scripted per tier.  Reference anchor: the budget discipline of
``mythril/support/model.py:25-49`` (a query gets at most its solver timeout).
"""
import time

from mythril_amd import search, workloads


class FakeEngine:
    def __init__(self, asm_raises=True, o3_ready_after=None, launch_s=0.0005, asm_ready_after=None,
                 jit_launch_s=None):
        self.asm_raises = asm_raises
        self.o3_ready_after = o3_ready_after
        self.asm_ready_after = asm_ready_after
        self.launch_s = launch_s
        self.jit_launch_s = jit_launch_s or {}  # handle kind -> seconds per candidate
        self.submits = {"asm": 0, "o3": 0}
        self.polls = {"asm": 0, "o3": 0}
        self.launches = {"interp": 0, "jit": 0}
        self.tickets = {}
        self.freed = []
        self.cancelled = []

    # program / generator handles
    def load(self, blob):
        return 11

    def load_gen(self, prog, blob):
        return 22

    def free(self, h):
        self.freed.append(("prog", h))

    def free_gen(self, h):
        self.freed.append(("gen", h))

    # compiles
    def jit_compile_async(self, prog, gh, asm=False):
        kind = "asm" if asm else "o3"
        self.submits[kind] += 1
        t = 100 + len(self.tickets)
        self.tickets[t] = (kind, time.perf_counter())
        return t

    def jit_poll(self, t):
        kind, at = self.tickets[t]
        self.polls[kind] += 1
        if kind == "asm" and self.asm_raises:
            raise RuntimeError("JIT assembly tier: op 16 outside the assembly tier")
        if kind == "asm" and self.asm_ready_after is not None and time.perf_counter() - at >= self.asm_ready_after:
            return 700 + t
        if kind == "o3" and self.o3_ready_after is not None and time.perf_counter() - at >= self.o3_ready_after:
            return 500 + t
        return None

    def jit_cancel(self, t):
        self.cancelled.append(t)

    def jit_free(self, h):
        self.freed.append(("jit", h))

    # launches: never a hit
    def search(self, prog, gh, seed, start, n, early_exit=True, assign=None):
        self.launches["interp"] += 1
        time.sleep(self.launch_s)
        return None, 0

    def jit_search(self, jh, seed, start, n, early_exit=True, assign=None):
        self.launches["jit"] += 1
        kind = "asm" if jh >= 700 else "o3"
        per = self.jit_launch_s.get(kind)
        time.sleep(n * per if per else self.launch_s)
        return None, 0


def _roots():
    return [c.raw for c in workloads.WORKLOADS["token_transfer_underflow"]()]


def test_refused_first_tier_is_submitted_once_when_o3_not_due():
    """ADVICE r4 (search.py): a first tier that refuses the program (Keccak, EXP, ...) while the O3
    kernel is not due (its expected compile exceeds the budget left) is asked once; before the fix
    it was resubmitted on every loop pass and kept interpreter launches at 1 ms."""
    eng = FakeEngine(asm_raises=True)
    res = search.search(eng, _roots(), timeout_s=0.08, max_candidates=1 << 40, jit_cost_s=10.0)
    assert res.index is None
    assert eng.submits == {"asm": 1, "o3": 0}
    assert eng.launches["interp"] > 3 and eng.launches["jit"] == 0
    assert res.engine == "interp"


def test_o3_still_replaces_interpreter_after_refused_first_tier():
    """With the O3 kernel due, a refused first tier does not stop the switch to the O3 kernel."""
    eng = FakeEngine(asm_raises=True, o3_ready_after=0.01)
    res = search.search(eng, _roots(), timeout_s=0.15, max_candidates=1 << 40, jit_cost_s=0.02)
    assert eng.submits == {"asm": 1, "o3": 1}
    assert eng.launches["jit"] > 0
    assert res.timing.get("jit_tier") == "o3"
    assert ("jit", 500 + 101) in eng.freed  # the O3 kernel's module released at the end


def test_tier_race_keeps_the_faster_first_tier():
    """When the O3 kernel arrives, one launch as large as the first tier's last decides which
    compiled kernel the search keeps: here the first tier is twice as fast, so it stays and the O3
    kernel is released at once."""
    eng = FakeEngine(asm_raises=False, asm_ready_after=0.005, o3_ready_after=0.03,
                     jit_launch_s={"asm": 1e-9, "o3": 2e-9})
    res = search.search(eng, _roots(), timeout_s=0.2, max_candidates=1 << 40, jit_cost_s=0.02)
    race = res.timing.get("tier_race")
    assert race is not None and race["kept"] == "asm", res.timing
    assert race["asm_rate"] > race["o3_rate"]
    assert res.timing.get("jit_tier") == "asm"
    assert ("jit", 500 + 101) in eng.freed  # the O3 kernel's module


def test_tier_race_switches_to_a_faster_o3():
    eng = FakeEngine(asm_raises=False, asm_ready_after=0.005, o3_ready_after=0.03,
                     jit_launch_s={"asm": 2e-9, "o3": 1e-9})
    res = search.search(eng, _roots(), timeout_s=0.2, max_candidates=1 << 40, jit_cost_s=0.02)
    race = res.timing.get("tier_race")
    assert race is not None and race["kept"] == "o3", res.timing
    assert res.timing.get("jit_tier") == "o3"
    assert ("jit", 700 + 100) in eng.freed  # the first tier's module
