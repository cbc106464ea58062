"""The plugin as Mythril finds it: installed, discovered through the entry point.

Mythril loads plugins only through installed entry points of the group ``mythril.plugins``
(``/root/reference/mythril/plugin/discovery.py:17-21``), builds those whose
``plugin_default_enabled`` is True (``discovery.py:45-58``, ``plugin/loader.py:73-80``), hands a
``MythrilLaserPlugin`` to ``LaserPluginLoader.load`` (``laser/plugin/loader.py:25-37``), and
``instrument_virtual_machine`` (``laser/plugin/loader.py:53-72``) calls the builder and
``initialize(laser)``.

This test installs the tree (``setup.cfg`` / ``pyproject.toml``) with pip into a temporary
prefix — offline, no dependencies, no build isolation — and then, in a fresh interpreter that
sees only that prefix and stand-in ``mythril`` modules with the reference's class shapes
(``plugin/interface.py:5-45``, ``laser/plugin/builder.py:7-21``, ``laser/plugin/interface.py:4-23``),
runs a restatement of that discovery and loading logic.  No GPU: the hook is installed, not
called.
"""
import json
import os
import shutil
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "mythril_amd"

STANDINS = {
    "mythril/__init__.py": "",
    "mythril/laser/__init__.py": "",
    "mythril/laser/plugin/__init__.py": "",
    # laser/plugin/interface.py:4-23
    "mythril/laser/plugin/interface.py": """
        class LaserPlugin:
            def initialize(self, symbolic_vm) -> None:
                raise NotImplementedError
    """,
    # laser/plugin/builder.py:7-21 (an ABC with an abstract __call__)
    "mythril/laser/plugin/builder.py": """
        from abc import ABC, abstractmethod
        from mythril.laser.plugin.interface import LaserPlugin

        class PluginBuilder(ABC):
            plugin_name = "Default Plugin Name"

            def __init__(self):
                self.enabled = True

            @abstractmethod
            def __call__(self, *args, **kwargs) -> LaserPlugin:
                pass
    """,
    "mythril/plugin/__init__.py": "",
    # plugin/interface.py:5-45: MythrilPlugin.__init__ does not chain to PluginBuilder.__init__
    "mythril/plugin/interface.py": """
        from abc import ABC
        from mythril.laser.plugin.builder import PluginBuilder as LaserPluginBuilder

        class MythrilPlugin:
            author = "Default Author"
            name = "Plugin Name"
            plugin_license = "All rights reserved."
            plugin_type = "Mythril Plugin"
            plugin_version = "0.0.1 "
            plugin_description = "This is an example plugin description"

            def __init__(self, **kwargs):
                pass

        class MythrilLaserPlugin(MythrilPlugin, LaserPluginBuilder, ABC):
            pass
    """,
    "mythril/support/__init__.py": "",
    "mythril/support/model.py": """
        def get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True):
            return "z3-model"
    """,
    "mythril/laser/ethereum/__init__.py": "",
    "mythril/laser/ethereum/state/__init__.py": "",
    "mythril/laser/ethereum/state/constraints.py": "from mythril.support.model import get_model\n",
    "mythril/analysis/__init__.py": "",
    "mythril/analysis/solver.py": """
        from mythril.support.model import get_model

        def _replace_with_actual_sha(concrete_transactions, model, code=None):
            return None
    """,
}

# What Mythril does with an installed plugin, restated from discovery.py:17-21,33-58,
# plugin/loader.py:41-80 and laser/plugin/loader.py:25-72.
DRIVER = """
import json, sys
import pkg_resources
import importlib.metadata as md
from mythril.plugin.interface import MythrilPlugin, MythrilLaserPlugin

# PluginDiscovery.init_installed_plugins (discovery.py:17-21)
installed = {ep.name: ep.load() for ep in pkg_resources.iter_entry_points("mythril.plugins")}
# the same group through importlib.metadata (what newer setuptools-free installs use)
md_names = sorted(ep.name for ep in md.entry_points(group="mythril.plugins"))
# PluginDiscovery.get_plugins(default_enabled=True) (discovery.py:45-58)
default_on = [n for n, c in installed.items() if c.plugin_default_enabled == True]
# PluginDiscovery.build_plugin (discovery.py:33-43)
cls = installed["mythgpu"]
assert issubclass(cls, MythrilPlugin), "not a MythrilPlugin"
plugin = cls(**{})
# MythrilPluginLoader.load (plugin/loader.py:41-60) -> _load_laser_plugin
assert isinstance(plugin, MythrilPlugin) and isinstance(plugin, MythrilLaserPlugin)
# LaserPluginLoader.load (laser/plugin/loader.py:25-37)
builders = {plugin.plugin_name: plugin}
# instrument_virtual_machine(vm, with_plugins=None) (laser/plugin/loader.py:53-72)
class VM:
    def __init__(self):
        self.hooks = {}
    def laser_hook(self, name):
        def deco(f):
            self.hooks.setdefault(name, []).append(f)
            return f
        return deco
vm = VM()
for name, b in builders.items():
    if not b.enabled:
        continue
    b(**{}).initialize(vm)

import mythril.support.model as mm, mythril.laser.ethereum.state.constraints as cm, mythril.analysis.solver as am
import mythril_amd, mythril_amd.plugin as mp, mythril_amd.native as nat
lib = nat.load_library()
print(json.dumps({
    "names": sorted(installed), "md_names": md_names, "default_on": default_on,
    "class": cls.__module__ + ":" + cls.__qualname__, "enabled": plugin.enabled,
    "have_mythril": mp.HAVE_MYTHRIL,
    "hooked": [getattr(m.get_model, "__wrapped_original__", None) is not None for m in (mm, cm, am)],
    "sha_hooked": am._replace_with_actual_sha is mp.batched_replace_with_actual_sha,
    "vm_hooks": sorted(vm.hooks),
    "pkg_file": mythril_amd.__file__, "lib": str(nat.LIB_PATH), "mg_version": lib.mg_version(),
}))
"""


def _write_standins(base: Path) -> None:
    for rel, text in STANDINS.items():
        p = base / rel
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(textwrap.dedent(text))


@pytest.fixture(scope="module")
def installed(tmp_path_factory):
    if not (PKG / "libmythgpu.so").exists():
        pytest.skip("libmythgpu.so not built (run __graft_entry__.build())")
    tmp = tmp_path_factory.mktemp("pkg")
    src = tmp / "src"
    # a copy of the distribution's files, so pip's in-tree build leaves the repository untouched
    (src / "mythril_amd").mkdir(parents=True)
    for name in ("setup.cfg", "pyproject.toml"):
        shutil.copy(ROOT / name, src / name)
    for p in PKG.iterdir():
        if p.suffix == ".py" or p.name in ("libmythgpu.so", "mythgpu_jitd"):
            shutil.copy2(p, src / "mythril_amd" / p.name)
    shutil.copytree(PKG / "smt", src / "mythril_amd" / "smt", ignore=shutil.ignore_patterns("__pycache__"))
    target = tmp / "site"
    r = subprocess.run([sys.executable, "-m", "pip", "install", "--no-deps", "--no-build-isolation", "--no-index",
                        "--disable-pip-version-check", "--target", str(target), str(src)],
                       capture_output=True, text=True, cwd=tmp, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    stand = tmp / "standins"
    _write_standins(stand)
    return tmp, target, stand


def test_install_ships_the_native_files(installed):
    _, target, _ = installed
    pkg = target / "mythril_amd"
    assert (pkg / "libmythgpu.so").stat().st_size > 0
    jitd = pkg / "mythgpu_jitd"
    assert jitd.exists() and os.access(jitd, os.X_OK), "the JIT helper must stay executable"
    assert (pkg / "smt" / "__init__.py").exists()
    (ep,) = list(target.glob("mythril_amd-*.dist-info/entry_points.txt"))
    text = ep.read_text()
    assert "[mythril.plugins]" in text and "mythgpu = mythril_amd.plugin:MythgpuPluginBuilder" in text


def test_discovery_builds_and_initializes_the_plugin(installed):
    tmp, target, stand = installed
    env = {k: v for k, v in os.environ.items() if k not in ("PYTHONPATH", "PYTHONHOME")}
    env["PYTHONPATH"] = os.pathsep.join([str(target), str(stand)])
    # cwd outside the repository: the installed copy is the one imported
    r = subprocess.run([sys.executable, "-c", DRIVER], capture_output=True, text=True, cwd=tmp, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["names"] == ["mythgpu"] and out["md_names"] == ["mythgpu"]
    assert out["default_on"] == ["mythgpu"]
    assert out["class"] == "mythril_amd.plugin:MythgpuPluginBuilder"
    assert out["enabled"] is True and out["have_mythril"] is True
    assert out["hooked"] == [True, True, True] and out["sha_hooked"] is True
    assert out["vm_hooks"] == ["stop_sym_exec"]
    assert Path(out["pkg_file"]).resolve().is_relative_to(target.resolve())
    assert Path(out["lib"]).resolve().is_relative_to(target.resolve())
    assert out["mg_version"] > 0
