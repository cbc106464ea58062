"""Build the C restatement ``oracle/libbveval.so`` (test infrastructure / CPU
baseline only).  Portable flags: the library travels to the GPU box host."""
import subprocess
from pathlib import Path

HERE = Path(__file__).resolve().parent
SRC = HERE / "bveval.c"
LIB = HERE / "libbveval.so"


def build(force: bool = False) -> Path:
    if not force and LIB.exists() and LIB.stat().st_mtime >= SRC.stat().st_mtime:
        return LIB
    tmp = LIB.with_suffix(".so.tmp")
    subprocess.run(["gcc", "-O3", "-std=c11", "-fopenmp", "-fPIC", "-shared", "-Wall", "-o", str(tmp), str(SRC)],
                   check=True)
    tmp.replace(LIB)
    return LIB


if __name__ == "__main__":
    print(build(force=True))
