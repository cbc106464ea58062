"""The eval-kernel roofline leg of bench.py on its own (for rocprofv3 passes, tools/profile_eval.sh):
usage: python tools/eval_probe.py <workload> [candidates] [reps] [asm 0|1] [tiled 0|1]
Prints one JSON line shaped like bench.py's (config.candidates_per_gpu_step, config.jit_source_sha16,
roofline.kernel_ms, value) so tools/pmc_summary.py can read it, plus the full eval record."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

import bench  # noqa: E402
from mythril_amd import native  # noqa: E402

w = sys.argv[1] if len(sys.argv) > 1 else "token_transfer_underflow"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 22
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
asm = len(sys.argv) > 4 and sys.argv[4] == "1"
tiled = len(sys.argv) > 5 and sys.argv[5] == "1"
torch.cuda.set_device(0)
eng = native.Engine.get()
r = bench.eval_roofline(eng, torch, w, n, str(ROOT / "profiles"), reps=reps, asm=asm, tiled=tiled)
print(json.dumps({"metric": "eval", "value": r["candidates_per_s"],
                  "config": {"candidates_per_gpu_step": n, "jit_source_sha16": r["jit_source_sha16"]},
                  "roofline": {"kernel_ms": r["kernel_ms"]}, "eval": r}), flush=True)
