"""Benchmark: candidate assignments evaluated / s on LASER path-constraint queries.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1
it is launched by torch.distributed.run, one rank per GPU.  Rank 0 prints ONE
JSON line.  ``--gpus N`` without a launcher (no ``WORLD_SIZE``) runs the product's own
multi-GPU path instead: one process opens N devices (``mg_init`` mask) and the shim splits
every search over them (``parallelism: inprocN``); it exits 2 if fewer than N GPUs are
visible.

A *step* is one full sweep of the hot path over one batch of candidates: every
rank evaluates C candidates of the workload's constraint program (no early exit:
every candidate is evaluated to its verdict) in the search kernel, then the ranks
agree on the lowest satisfying index with one RCCL all-reduce(MIN) over xGMI —
the only exchange step the path has.  Candidate shards are disjoint index ranges
(weak scaling).  Inputs are generated on the device (nothing crosses PCIe inside
the timed region).

roofline: achieved = VALU lane-instructions per candidate MEASURED by rocprofv3
(SQ_INSTS_VALU x 64 / candidates, committed under profiles/ by tools/profile.sh and
matched to this exact kernel by the SHA of its JIT source) x C / the search kernel's
mean duration (HIP events on the engine's own stream); peak = INT32 VALU lane-ops/s
of MI355X (256 CU x 4 SIMD x 32 lanes x 2.4 GHz), so frac <= 1 by construction.  The
SURVEY §8(d) cost-table figure (program.cpp op_cost) is reported beside it as
``algorithmic``: it prices work the JIT folds away, so it is not a roofline.
cpu_baseline: the plain-C restatement (oracle/bveval.c, OpenMP) timed on the
host cores over a bounded sample of the same candidates (rank 0, N == 1).
"""
import argparse
import glob
import hashlib
import json
import os
import re
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12  # 78.6 T int32 lane-ops/s
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
METRIC = "candidate assignments evaluated/sec (node) + time-to-first-model vs z3"
# workload -> the BASELINE.json config it stands for
CONFIG_OF = {
    "suicide_kill": "C1 suicide_kill -t 2 (BASELINE.json configs[0] query shape; GPU stand-in for the z3 run)",
    "token_transfer_underflow": "C2 token_transfer_underflow (BASELINE.json configs[1])",
    "etherstore_reentrancy": "C2 etherstore_reentrancy (BASELINE.json configs[1])",
    "bectoken_batch_overflow": "C3 bectoken_batch_overflow (BASELINE.json configs[2])",
    "walletlibrary_kill": "C4 walletlibrary_kill -t 3 (BASELINE.json configs[3])",
    "sha3_keyed_mapping": "C5 sha3_keyed_mapping (BASELINE.json configs[4])",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="token_transfer_underflow")
    ap.add_argument("--candidates", type=int, default=1 << 30,
                    help="candidates per GPU per step (~6 ms on C2: SURVEY §8(e) sizes an epoch at 5-10 ms "
                         "per GPU, so the per-step host sync and the RCCL exchange stay ~1 %% of a step "
                         "at 8 GPUs)")
    ap.add_argument("--seed", type=int, default=0x6D797468)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-stream", action="store_true", help="skip the LASER-shaped get_model stream")
    ap.add_argument("--no-ttfm", action="store_true",
                    help="skip the time-to-first-model searches (profiling passes: full launches only)")
    ap.add_argument("--no-eval", action="store_true", help="skip the eval-kernel roofline (roofline_eval)")
    ap.add_argument("--eval-candidates", type=int, default=1 << 22,
                    help="candidates per eval launch (HBM-resident SoA; C2: 1,241 B each)")
    ap.add_argument("--eval-only", action="store_true",
                    help="profiling pass: only the eval-kernel launches (tools/profile.sh eval)")
    ap.add_argument("--engine", choices=["jit", "asm", "interp"], default="jit",
                    help="jit: the O3 query kernel (clang + LLVM through comgr); asm: the JIT's first tier "
                         "(gfx950 assembly emitted by the engine); interp: the generic interpreter kernel")
    ap.add_argument("--o3-only", action="store_true",
                    help="--engine jit: time the O3 kernel even where the first tier is faster")
    ap.add_argument("--pmc-dir", default=str(ROOT / "profiles"),
                    help="where tools/profile.sh summaries (pmc_<workload>*.json) are looked up by kernel SHA")
    return ap.parse_args()


def load_pmc(pmc_dir: str, workload: str, sha: str, candidates: int):
    """The committed rocprofv3 summary of THIS kernel (same JIT source SHA, same launch size)."""
    for f in sorted(glob.glob(os.path.join(pmc_dir, f"*pmc*{workload}*.json")), reverse=True):
        try:
            d = json.loads(Path(f).read_text())
        except (OSError, ValueError):
            continue
        if d.get("jit_source_sha16") == sha and d.get("candidates_per_launch") == candidates:
            d["_file"] = os.path.relpath(f, ROOT)
            return d
    return None


def main():
    args = parse()
    # code objects left on disk by an earlier process (tests, a previous bench) would hide the
    # compile in the cold numbers: the engine's on-disk code-object cache is off for the bench
    os.environ.setdefault("MYTHGPU_JIT_DISK_CACHE", "0")
    # stdout carries exactly the one JSON line: native libraries print to fd 1 on their own
    # (RCCL's version banner at communicator set-up), so fd 1 goes to stderr for the run and the
    # line is written to the saved stdout
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # torch first: its HIP runtime is the one process-wide runtime the engine then shares
    import torch
    import torch.distributed as dist

    # launched by torch.distributed.run (even at one rank): use the RCCL exchange path
    distributed = world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
    # --gpus N without a launcher: the product's own multi-GPU path — one process opens N devices
    # (mg_init mask) and every search call is split over them inside the shim, host min/sum
    inproc = 1
    if not distributed and args.gpus > 1:
        visible = torch.cuda.device_count()
        if visible < args.gpus:
            print(f"bench.py: --gpus {args.gpus} but only {visible} GPU(s) visible", file=sys.stderr)
            sys.exit(2)
        inproc = args.gpus
        os.environ["MYTHGPU_DEVICES"] = ",".join(str(d) for d in range(inproc))
    torch.cuda.set_device(local_rank)
    if distributed:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    from mythril_amd import build, native, search, ssa, workloads

    if rank == 0 and not native.LIB_PATH.exists():
        build.build()
    if distributed:
        dist.barrier()
    os.environ["MYTHGPU_DEVICE"] = str(local_rank)
    eng = native.Engine.get()
    if eng.n_devices != inproc:
        print(f"bench.py: engine opened {eng.n_devices} device(s), wanted {inproc}", file=sys.stderr)
        sys.exit(2)

    cs = workloads.WORKLOADS[args.workload]()
    roots = [c.raw for c in cs]
    # the program and generator the product path (search.search / the get_model hook) runs
    P, blob = search.prepare(roots)
    prog = eng.load(P.to_bytes())
    info = eng.info(prog)
    gh = eng.load_gen(prog, blob)
    C = args.candidates
    jit = None
    compile_ms = None
    sha = None
    if args.engine == "asm":
        sha = hashlib.sha256(native.jit_asm(P.to_bytes(), blob).encode()).hexdigest()[:16]
        t1 = time.perf_counter()
        jit = eng.jit_compile(prog, gh, asm=True)
        compile_ms = (time.perf_counter() - t1) * 1e3
    if args.engine == "jit":
        sha = hashlib.sha256(native.jit_source(P.to_bytes(), blob).encode()).hexdigest()[:16]
        # cold compile: comgr's on-disk cache and the engine's code-object cache off, so a
        # kernel compiled by an earlier process (tests, a previous bench) is not reported as a
        # compile cost
        prev = {k: os.environ.get(k) for k in ("AMD_COMGR_CACHE", "MYTHGPU_JIT_DISK_CACHE")}
        os.environ.update({k: "0" for k in prev})
        jit = eng.jit_compile(prog, gh)
        for k, v in prev.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v
        compile_ms = eng.jit_info(jit)[0]

    from mythril_amd.distributed import chunk_start, first_hit_allreduce

    # --engine jit: the engine's faster compiled tier for this query, as search.search races them (the
    # first tier beats the O3 kernel on some queries): one untimed step of each after the warm-up
    tier = "o3" if args.engine == "jit" else ("asm" if args.engine == "asm" else None)
    tier_rates = None
    jit_o3 = None
    if args.engine == "jit" and not args.o3_only:
        try:
            ja_h = eng.jit_compile(prog, gh, asm=True)
        except native.EngineUnsupported:
            ja_h = None
        if ja_h is not None:
            cc0 = C * inproc
            rates = {}
            for name, h in (("o3", jit), ("asm", ja_h)):
                for _ in range(max(1, args.warmup)):
                    eng.jit_search(h, args.seed, chunk_start(0, rank, world, cc0), cc0, early_exit=False)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                eng.jit_search(h, args.seed, chunk_start(1, rank, world, cc0), cc0, early_exit=False)
                torch.cuda.synchronize()
                rates[name] = cc0 / (time.perf_counter() - t1)
            r_t = torch.tensor([rates["o3"], rates["asm"]], dtype=torch.float64, device="cuda")
            if distributed:  # every rank takes the same tier: the slowest rank's view decides
                dist.all_reduce(r_t, op=dist.ReduceOp.MIN)
            tier_rates = {"o3": float(r_t[0].item()), "asm": float(r_t[1].item())}
            if tier_rates["asm"] > tier_rates["o3"]:
                jit_o3 = jit  # kept for the first tier's agreement check below
                jit, tier = ja_h, "asm"
                sha = hashlib.sha256(native.jit_asm(P.to_bytes(), blob).encode()).hexdigest()[:16]
            else:
                eng.jit_free(ja_h)

    # in-process multi-GPU: one call sweeps inproc x C candidates, split over the devices in the shim
    CC = C * inproc

    def step(s):
        start = chunk_start(s, rank, world, CC)
        if jit is not None:
            idx, nh = eng.jit_search(jit, args.seed, start, CC, early_exit=False)
        else:
            idx, nh = eng.search(prog, gh, args.seed, start, CC, early_exit=False)
        if distributed:  # the path's one exchange step: all-reduce(MIN) of the first hit over RCCL
            idx = first_hit_allreduce(idx, device="cuda")
        return idx, nh

    for s in range(args.warmup):
        step(s)
    eng.reset_stats()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    total_hits = 0
    for s in range(args.warmup, args.warmup + args.steps):
        _, nh = step(s)
        total_hits += nh
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    dt = time.perf_counter() - t0
    st = eng.stats()
    kernel_ms = st.kernel_ms_total / max(st.launches, 1)
    dt_t = torch.tensor([dt], dtype=torch.float64, device="cuda")
    km_t = torch.tensor([kernel_ms], dtype=torch.float64, device="cuda")
    if distributed:
        dist.all_reduce(dt_t, op=dist.ReduceOp.MAX)
        dist.all_reduce(km_t, op=dist.ReduceOp.MAX)
    dt = float(dt_t.item())
    kernel_ms = float(km_t.item())

    # the JIT's first tier (gfx950 assembly emitted by the engine, jit_asm.cpp): its cold compile (comgr's
    # cache off) and its rate at 2^28 candidates per launch on this workload; the product runs it from a
    # few ms after a query's first miss until the O3 kernel above is ready
    asm_tier = None
    if rank == 0 and args.engine == "jit" and not args.no_ttfm:
        prev_cc = os.environ.get("AMD_COMGR_CACHE")
        os.environ["AMD_COMGR_CACHE"] = "0"
        t1 = time.perf_counter()
        try:
            ja = eng.jit_compile(prog, gh, asm=True)
            asm_tier = {"compile_ms_cold": (time.perf_counter() - t1) * 1e3}
        except native.EngineUnsupported as e:
            ja, asm_tier = None, {"unsupported": str(e)}
        if prev_cc is None:
            os.environ.pop("AMD_COMGR_CACHE")
        else:
            os.environ["AMD_COMGR_CACHE"] = prev_cc
        if ja is not None:
            na = 1 << 28
            eng.jit_search(ja, args.seed, 0, na, early_exit=False)
            eng.reset_stats()
            for s_ in range(4):
                eng.jit_search(ja, args.seed, (s_ + 1) * na, na, early_exit=False)
            st_a = eng.stats()
            km_a = st_a.kernel_ms_total / max(st_a.launches, 1)
            o3h = jit_o3 if jit_o3 is not None else jit
            o3 = eng.jit_search(o3h, args.seed, na, na, early_exit=False) if o3h is not None else None
            asm_tier.update({"candidates_per_launch": na, "kernel_ms": km_a, "candidates_per_s": na / (km_a * 1e-3),
                             "agrees_with_o3_on_a_launch": o3 == eng.jit_search(ja, args.seed, na, na,
                                                                                early_exit=False)})
            eng.jit_free(ja)

    # time to first model (early-exit search from index 0 + model read-back), rank 0 only
    ttfm_ms = None
    ttfm_breakdown = None
    ttfm_cold_ms = None
    ttfm_cold_breakdown = None
    if rank == 0 and not args.no_ttfm:
        # cold: a fresh flatten cache (the query is new to the process), nothing pooled for it yet
        from mythril_amd import ssa as _ssa

        search.FLATTEN_CACHE = _ssa.FlattenCache(aux_words=True)
        search._GEN_CACHE.clear()
        eng.cache_clear()
        t1 = time.perf_counter()
        res_cold = search.search(eng, roots, seed=args.seed, max_candidates=1 << 30, timeout_s=30)
        ttfm_cold_ms = (time.perf_counter() - t1) * 1e3
        ttfm_cold_breakdown = {k: round(v, 3) for k, v in res_cold.timing.items()}
        # warm: the median of 7 repeats (one query is ~1 ms of host + GPU work, so a single
        # sample is at the mercy of host scheduling); the breakdown is the median run's
        runs = []
        for _ in range(7):
            t1 = time.perf_counter()
            res = search.search(eng, roots, seed=args.seed, max_candidates=1 << 30, timeout_s=30)
            runs.append(((time.perf_counter() - t1) * 1e3, res))
        runs.sort(key=lambda r: r[0])
        ms, res = runs[len(runs) // 2]
        ttfm_ms = ms if res.index is not None else None
        ttfm_breakdown = {k: round(v, 3) for k, v in res.timing.items()}
        ttfm_breakdown["engine"] = res.engine
        ttfm_breakdown["warm_runs"] = len(runs)

    # time to first model of a query that needs a search: the workload plus a ~2^-24 needle on one of
    # its own 256-bit symbols (Extract(23, 0, v * K) == C), through the product path search.search
    # (interpreter first, async JIT compile, compiled kernel); "cold" compiles the kernel inside the
    # timing, "warm" finds it in the code cache (the same query asked again)
    hard = None
    if rank == 0 and not args.no_ttfm:
        hroots = hard_query(cs, HARD_BITS.get(args.workload, 24))
        search.FLATTEN_CACHE = ssa.FlattenCache(aux_words=True)
        search._GEN_CACHE.clear()
        eng.cache_clear()
        hard = {}
        for label in ("cold", "warm"):
            t1 = time.perf_counter()
            rh = search.search(eng, hroots, seed=args.seed, max_candidates=1 << 36, timeout_s=20)
            hard[f"{label}_ms"] = (time.perf_counter() - t1) * 1e3
            hard[f"{label}_engine"] = rh.engine
            hard["index"] = rh.index
            hard["candidates"] = rh.scanned
            if label == "cold":
                hard["jit_compile_ms"] = rh.timing.get("jit_compile_ms")
            hard[f"{label}_timing"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in rh.timing.items()}
        hb = HARD_BITS.get(args.workload, 24)
        hard["needle"] = f"Extract({hb - 1}, 0, x * K) == C on a fresh 256-bit symbol x (~2^-{hb} per candidate)"

    # time to first model on ALL ranks: the compiled kernel sweeps epochs of `chunk` candidates per
    # rank from index 0, one all-reduce(MIN) per epoch (distributed.sharded_first_hit); the index found
    # is the global lowest, identical at every GPU count
    from mythril_amd.distributed import sharded_first_hit

    def first_hit(start, count):
        if jit is not None:
            return eng.jit_search(jit, args.seed, start, count, early_exit=True)[0]
        return eng.search(prog, gh, args.seed, start, count, early_exit=True)[0]

    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if args.no_ttfm:
        ttfm_index = None
    elif distributed:
        ttfm_index, _ = sharded_first_hit(first_hit, rank, world, 1 << 20, max_epochs=1024, device="cuda")
    else:
        ttfm_index = None
        for e in range(1024):
            ttfm_index = first_hit(e * inproc << 20, inproc << 20)
            if ttfm_index is not None:
                break
    ttfm_sharded_ms = (time.perf_counter() - t1) * 1e3 if ttfm_index is not None else None

    # the drop-in under a LASER-shaped stream of this workload's queries through solver.get_model,
    # 200 ms budget each (tools/stream_bench.py; async JIT compile inside the budget), rank 0
    stream = None
    if rank == 0 and world == 1 and inproc == 1 and not args.no_stream:
        sys.path.insert(0, str(Path(__file__).resolve().parent / "tools"))
        import stream_bench

        rows, summ = stream_bench.run([args.workload], 200.0, quiet=True)
        r0 = rows[0]
        # indices scanned per second, NOT a throughput of full evaluations: the early-exit search stops
        # a wave at the first constraint all 64 of its candidates fail, and those indices count as scanned
        stream = {"queries": r0["queries"], "budget_ms": 200.0, "stream_s": r0["stream_s"],
                  "scan_rate_incl_early_exit": r0["stream_rate"],
                  "budget_bound_scan_rate_incl_early_exit": r0["budget_bound_rate"],
                  "engines": r0["engines"], "jit_compile_s_avg": summ["jit_compile_s_avg"],
                  "note": "indices scanned/s through solver.get_model incl. flatten, async compile, model read-back; "
                          "waves rejected by an early constraint stop there (early exit), so this is not comparable "
                          "with `value` (every candidate evaluated in full)"}
        # the same stream through the hook's race core against a z3 stand-in answering unsat after 50 ms:
        # what a GPU miss adds to z3's own time (plugin.race; no z3 on the box)
        rr = stream_bench.run_race([args.workload], 200.0, 50.0, quiet=True)[0]
        stream["race"] = {k: rr[k] for k in ("race_z3_standin_ms", "gpu_won", "z3_won", "added_ms_per_miss_median",
                                             "added_ms_per_miss_max", "gpu_won_wall_ms_median")}

    # the eval kernel's own roofline (unspecialised C2 and C4 programs on HBM-resident SoA inputs)
    evals = None
    if rank == 0 and world == 1 and inproc == 1 and not args.no_eval:
        evals = []
        # the O3 and first-tier (jit_asm.cpp) eval kernels, each on the [row][candidate] SoA and on the
        # tiled SoA (MG_JIT_SOA_TILED: a group's rows in one block)
        # (tiled SoA: a group's rows in one block); then the tier the engine picks when none is named
        # (mg_jit_compile_ex without MG_JIT_ASM / MG_JIT_O3: what batched Model.eval gets by default)
        for etier in ("o3", "asm", "default"):
            for tiled in (False, True):
                for w in EVAL_WORKLOADS:
                    try:
                        evals.append(eval_roofline(eng, torch, w, args.eval_candidates, args.pmc_dir, tiled=tiled,
                                                   tier=etier))
                    except native.EngineUnsupported as e:
                        evals.append({"workload": CONFIG_OF[w], "tier_requested": etier,
                                      "kernel": eval_kernel_name(etier == "asm", tiled), "unsupported": str(e)})

    # CPU baseline: the C restatement over a bounded sample of the same candidates
    cpu = None
    if rank == 0 and world == 1 and inproc == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(P, blob, args, eng, prog, gh, jit, tier)

    if rank == 0:
        total = world * inproc * C * args.steps
        value = total / dt
        kernel_s = kernel_ms * 1e-3
        pmc = load_pmc(args.pmc_dir, args.workload, sha, C) if sha else None
        roofline = {"bound": "valu", "achieved": None, "peak": VALU_PEAK_TOPS, "unit": "TOP/s (int32 lane-ops)",
                    "frac": None, "traffic": None, "kernel_ms": kernel_ms,
                    "basis": "no rocprofv3 summary for this kernel under profiles/ (run tools/profile.sh)"}
        if pmc is not None:
            n_instr = pmc["derived"]["valu_wave_instructions_per_candidate"]
            achieved = n_instr * C / kernel_s / 1e12
            roofline.update(achieved=achieved, frac=achieved / VALU_PEAK_TOPS,
                            traffic=pmc["derived"].get("hbm_bytes_per_launch"),
                            valu_instructions_per_candidate=n_instr,
                            basis=f"measured VALU lane-instructions per candidate ({pmc['_file']}, "
                                  f"rocprofv3 SQ_INSTS_VALU) x candidates / kernel time")
        algorithmic = {"limb_ops_per_candidate": int(info.limb_ops),
                       "achieved_T": info.limb_ops * C / kernel_s / 1e12,
                       "note": "SURVEY §8(d) fixed cost table; prices work the JIT folds (Concat/Extract look-through, "
                               "range-decided compares), so it is not a roofline fraction"}
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "candidate assignments/s",
            "n_gpus": world * inproc,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": dt / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (device-generated candidates of a LASER-shaped query; no solc/z3 in image)",
            "config": {
                "workload": CONFIG_OF[args.workload],
                "candidates_per_gpu_step": C,
                "program_instrs": int(info.n_instrs),
                "coords": int(info.n_coords),
                "engine": args.engine,
                "jit_source_sha16": sha,
                "jit_tier": tier,
                "jit_tier_rates": tier_rates,
                "jit_compile_ms_cold": compile_ms,
                "parallelism": f"inproc{inproc}" if inproc > 1 else f"shard{world}",
            },
            "roofline": roofline,
            "roofline_eval": evals,
            "algorithmic": algorithmic,
            "cpu_baseline": cpu,
            "time_to_first_model_ms": ttfm_ms,
            "time_to_first_model_cold_ms": ttfm_cold_ms,
            "time_to_first_model_cold_breakdown": ttfm_cold_breakdown,
            "time_to_first_model_breakdown": ttfm_breakdown,
            "time_to_first_model_sharded_ms": ttfm_sharded_ms,
            "first_model_index": ttfm_index,
            "time_to_first_model_hard_ms": None if hard is None else hard["cold_ms"],
            "time_to_first_model_hard": hard,
            "jit_asm_tier": asm_tier,
            "hits_in_timed_region": int(total_hits),
            "hit_rate_in_timed_region": total_hits / total,
            "dropin_stream": stream,
        }
        os.write(out_fd, (json.dumps(out) + "\n").encode())
    if jit is not None:
        eng.jit_free(jit)
    eng.free_gen(gh)
    eng.free(prog)
    if distributed:
        dist.destroy_process_group()


EVAL_WORKLOADS = ("token_transfer_underflow", "walletlibrary_kill")


def eval_kernel_name(asm, tiled):
    return ("mgj_eval first tier (asm)" if asm else "mgj_eval (unspecialised program)") + (", tiled SoA" if tiled else "")


def eval_roofline(eng, torch, workload, n, pmc_dir, reps=5, asm=False, tiled=False, tier=None):
    """``Model.eval`` batched (``laser/smt/model.py:45-59``): the compiled eval kernel
    (``mg_jit_eval_dev``) of the UNSPECIALISED program — no generator, no value ranges, every
    instruction evaluated — over n candidates whose coordinates are already in HBM as a
    ``[coord limb row][candidate]`` uint32 SoA (uniform random, masked to each coordinate's
    width), one verdict byte out per candidate.  Algorithmic bytes per candidate: 4 x the SoA
    rows the program reads (a coordinate the program never reads — an AUX word whose bytes
    it reads through its sites, a lazy site — is not fetched) + 1 verdict byte out.

    ``tier``: "o3" / "asm" ask for a tier (MG_JIT_O3 / MG_JIT_ASM), "default" asks for none — the
    engine then picks per program (engine.hip eval_tier_pick_asm) and the entry says which it built;
    None: ``asm`` decides, as before."""
    from mythril_amd import native, search, ssa, workloads

    cs = workloads.WORKLOADS[workload]()
    P, _ = search.prepare([c.raw for c in cs])
    # verdicts only (mg_jit_eval_dev without a watch buffer): the program without the model
    # watch rows, whose eval kernel walks the SoA rows with one pointer (jit.cpp K_COORD)
    prev = P.watch
    P.set_watch([])
    blob = P.to_bytes()
    P.set_watch(prev)
    prog = eng.load(blob)
    info = eng.info(prog)
    if tier is None:
        tier = "asm" if asm else "o3"
    try:
        jh = eng.jit_compile(prog, 0, asm=tier == "asm", o3=tier == "o3", tiled=tiled)
        asm = bool(eng.jit_layout(jh)[0] & native.MG_JIT_ASM)
    except Exception:
        eng.free(prog)
        raise
    try:
        cw = int(info.coord_words)
        mask = np.zeros(cw, dtype=np.int64)
        offs = P.coord_row_offsets()
        for c in P.coords:
            for j in range(ssa.limbs(c.width)):
                bits = min(32, c.width - 32 * j)
                mask[offs[c.index] + j] = (1 << bits) - 1
        soa = torch.randint(-(1 << 31), (1 << 31) - 1, (cw, n), dtype=torch.int32, device="cuda")
        soa &= torch.from_numpy(mask.astype(np.uint32).view(np.int32)).to("cuda")[:, None]
        if tiled:
            soa = native.tile_soa(soa)
        ver = torch.empty(n, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        eng.jit_eval_dev(jh, soa.data_ptr(), n, ver.data_ptr())  # warm-up (module load, caches)
        eng.reset_stats()
        for _ in range(reps):
            eng.jit_eval_dev(jh, soa.data_ptr(), n, ver.data_ptr())
        st = eng.stats()
        kernel_ms = st.kernel_ms_total / max(st.launches, 1)
        sat = int(ver.sum().item())
        src = native.jit_asm(blob, tiled=tiled) if asm else native.jit_source(blob, tiled=tiled)
        sha = hashlib.sha256(src.encode()).hexdigest()[:16]
        rows_read = len(set(re.findall(r"soa\[\(uint64_t\)(\d+)u \* n \+ i\]|// soa row (\d+)|; soa row (\d+)", src)))
    finally:
        eng.jit_free(jh)
        eng.free(prog)
    del soa, ver
    bpc = 4 * rows_read + 1
    gbs = n * bpc / (kernel_ms * 1e-3) / 1e9
    out = {"workload": CONFIG_OF[workload], "tier_requested": tier, "tier_built": "asm" if asm else "o3",
           "kernel": eval_kernel_name(asm, tiled), "soa_layout": "tiled" if tiled else "row-major", "candidates_per_launch": n,
           "program_instrs": int(info.n_instrs), "coord_words": cw, "soa_rows_read": rows_read,
           "bytes_per_candidate": bpc,
           "kernel_ms": kernel_ms, "candidates_per_s": n / (kernel_ms * 1e-3),
           "hbm": {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS},
           "valu": None, "traffic": None, "sat_fraction": sat / n, "jit_source_sha16": sha}
    pmc = load_pmc(pmc_dir, ("evalasm_" if asm else "eval_") + ("tiled_" if tiled else "") + workload, sha, n)
    if pmc is not None:
        n_instr = pmc["derived"]["valu_wave_instructions_per_candidate"]
        achieved = n_instr * n / (kernel_ms * 1e-3) / 1e12
        out["valu"] = {"achieved": achieved, "peak": VALU_PEAK_TOPS, "unit": "TOP/s (int32 lane-ops)",
                       "frac": achieved / VALU_PEAK_TOPS, "valu_instructions_per_candidate": n_instr,
                       "basis": pmc["_file"]}
        out["traffic"] = pmc["derived"].get("hbm_bytes_per_launch")
    out["bound"] = "hbm" if out["valu"] is None or out["hbm"]["frac"] >= out["valu"]["frac"] else "valu"
    return out


# needle bits of the hard query per workload: 24 (~2^-24) on top of the C1-C4 queries, which their
# generators satisfy often; C5 itself holds about 1 candidate in 2^17, so its needle
# is 8 bits: ~2^25 candidates to the first model either way
HARD_BITS = {"sha3_keyed_mapping": 8}


def hard_query(cs, bits: int = 24):
    """The workload's constraints plus a ~2^-bits needle: ``Extract(bits-1, 0, x * K) == C`` on a
    fresh 256-bit symbol ``x`` (a path symbol would inherit the generator's dictionaries, which may
    never reach the needle), so about one candidate in 2^bits of the workload's satisfying ones
    satisfies the query."""
    from mythril_amd.smt import Extract, symbol_factory

    x = symbol_factory.BitVecSym("hard_x", 256)
    k = symbol_factory.BitVecVal(0x9E3779B97F4A7C15F39CC0605CEDC835, 256)
    needle = Extract(bits - 1, 0, x * k) == symbol_factory.BitVecVal(0xA5C3E1 & ((1 << bits) - 1), bits)
    return [c.raw for c in cs] + [needle.raw]


def cpu_baseline(P, blob, args, eng, prog, gh, jit=None, tier=None):
    from oracle import cport

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    start = 1 << 40  # a window the GPU also evaluates below
    n = 4096
    t = time.perf_counter()
    cport.search(P.to_bytes(), blob, args.seed, start, n, threads=threads)
    dt = time.perf_counter() - t
    n = int(min(max(n, n * args.cpu_seconds / max(dt, 1e-6)), 1 << 26))
    t = time.perf_counter()
    first, hits, _ = cport.search(P.to_bytes(), blob, args.seed, start, n, threads=threads)
    dt = time.perf_counter() - t
    g_first, g_hits = eng.search(prog, gh, args.seed, start, n, early_exit=False)
    if jit is not None:
        assert eng.jit_search(jit, args.seed, start, n, early_exit=False) == (g_first, g_hits)
    # per-candidate verdicts on the first 2^16 of the window: the timed tier's own kernels built with
    # mgj_gen (one verdict byte per candidate) against the C port's, byte for byte
    nv = min(n, 1 << 16)
    _, _, want = cport.search(P.to_bytes(), blob, args.seed, start, nv, threads=threads, verdicts=True)
    if tier in ("asm", "o3"):
        jv = eng.jit_compile(prog, gh, gen_verdicts=True, asm=tier == "asm")
        try:
            got = eng.jit_verdicts(jv, args.seed, start, nv)
        finally:
            eng.jit_free(jv)
    else:
        got, _ = eng.eval_generated(prog, gh, args.seed, start, nv)
    per_candidate = bool(np.array_equal(np.asarray(got, dtype=np.uint8), np.asarray(want, dtype=np.uint8)))
    return {
        "value": n / dt,
        "unit": "candidate assignments/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{n} candidates [{start}, {start + n}) of the same workload/seed; {dt:.1f} s",
        "agrees_with_gpu": bool(first == g_first and hits == g_hits),
        "verdicts_checked": nv,
        "verdicts_agree": per_candidate,
        "verdicts_kernel": f"mgj_gen ({tier} tier)" if tier in ("asm", "o3") else "k_run (interpreter)",
    }


if __name__ == "__main__":
    main()
