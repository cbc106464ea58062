"""The JIT compiler runs in its own process (mythgpu_jitd): a compiler abort must not take the
caller down (SURVEY §5 "Failure detection": never raise a new exception type into LASER).
``MYTHGPU_JITD_FAULT=abort`` makes the helper abort() on a request, standing in for an LLVM
``report_fatal_error``.  Each case runs in a child process, since the abort turns the JIT off
for the process that sees it."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

SCRIPT = Path(__file__).resolve().parent / "scripts" / "jit_fault_probe.py"


def _run(mode):
    r = subprocess.run([sys.executable, str(SCRIPT), mode], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1]), r.stderr


def test_compiler_abort_is_contained_host():
    out, err = _run("host")
    assert out["pid_before"] > 0  # compiled in the helper, not in this process
    assert "killed by signal 6" in out["fault_error"]  # the abort reached only the helper
    assert "JIT is off" in out["after_error"]  # no restart: later compiles fail at once
    assert out["pid_after"] == -2
    assert "killed by signal 6" in err


@pytest.mark.gpu
def test_compiler_abort_search_continues_on_interpreter():
    out, _ = _run("gpu")
    assert out["ref"] is not None
    assert out["always"] == out["auto"] == out["ref"], out  # same first hit, found on k_run
    assert out["engines"] == ["interp", "interp"] and out["pid_after"] == -2 and out["model_ok"]
