#!/usr/bin/env python3
"""Headline benchmark: simulator throughput (sim KIPS, whole node) on the
Rodinia-2.0-ft suite (synthetic traces of the suite's shape) with the GV100
config (BASELINE.json config #2: SM7_GV100 = the SM7_QV100 gpgpusim.config at
1447 MHz, plus the SM7_QV100 trace.config), one simulated GPU per MI355X.

One "step" = every application of the suite simulated end to end (trace load
+ coalescing + cycle simulation + stats), followed -- when N > 1 -- by the
suite's closing all-reduce (examples/all-reduce) whose completion is
synchronised across the N simulated GPUs over RCCL.  Weak scaling: every rank
simulates its own GPU running the full suite.

Engines: ``node`` (default with a GPU) runs each application on the engine that
minimises the step's makespan -- the HIP cycle engine on the MI355X for
applications with much parallel work per epoch, the CPU engine on the rank's
share of host cores for latency-bound ones (placement measured during warmup,
parallel/multi_gpu.py DistributedSuite.plan).  ``gpu`` / ``cpu`` force one
engine (``cpu``: one single-threaded simulation per core, the reference's
job-level parallelism).

    python bench.py --gpus N --steps K --warmup W
Rank 0 prints ONE JSON line.  KIPS = simulated thread instructions (the
reference's gpu_tot_sim_insn, shader.cc:1911) of all ranks / wall seconds /
1000; the baseline is the reference's published 349 KIPS (heartwall,
util/job_launching/README.md:77).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time



def _gpu_env(sweep: bool) -> None:
    """GPU-engine settings, applied before the process's first HIP call.
    Hardware queues: one kernel per in-flight simulation, and kernels of
    streams sharing a queue run one after another
    (accel_sim_framework_distributed_amd/__init__.py).  The sweep is a
    throughput job (16 configurations x 10 apps): there the split build runs
    two engine waves per SIMD (ASIM_GPU_SPLIT_WAVES=2, engine_k_split2.hip),
    16 simulations in flight on 16 queues -- sweep GPU engine 50.3k -> 55.3k
    sim KIPS on one box, while the 11-app suite, whose 11 simulations never
    fill the GPU, is faster at one wave per SIMD (63.1k vs 60.0k)
    (profiles/r6/README.md, "Two engine waves per SIMD")."""
    if sweep:
        os.environ.setdefault("ASIM_GPU_SPLIT_WAVES", "2")
        os.environ.setdefault("ASIM_GPU_HW_QUEUES", "16")
    want = int(os.environ.get("ASIM_GPU_HW_QUEUES", "8") or 0)
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < want:
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, want))

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_KIPS = 349.0


def _parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="GV100")
    ap.add_argument("--engine", default="auto", choices=["auto", "node", "gpu", "cpu"])
    ap.add_argument("--apps", default="all")
    ap.add_argument("--trace-dir", default=None)
    ap.add_argument("--verbose", action="store_true")
    # "nccl" (RCCL over xGMI) is the production path; "gloo" lets several ranks
    # share one card to rehearse the multi-rank GPU-engine path on a 1-GPU box
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "nccl", "gloo"])
    # BASELINE.json config #5: every app x the tuner's 16 search configs, one
    # batch of independent simulations per step (parallel/sweep.py)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--sweep-configs", type=int, default=16)
    return ap.parse_args()


def _cycle_mae():
    """The latest committed MI355X cycle correlation, labelled as what it is:
    an offline run, NOT measured by this bench run (tools/gpu_correlate.sh:
    the Rodinia-2.0-ft HIP suite traced by the automatic ISA tracer, timed
    with rocprofv3, simulated by the MI355X cycle engine with the tuned
    MI355X config; correlator semantics of plot-correlation.py)."""
    # the latest full GPU correlation run (fresh ubench -> tuner -> traces ->
    # timings -> counters on one box): profiles/correlation/LATEST names it
    # (tools/gpu_correlate.sh records; updated with every committed run)
    cdir = os.path.join(ROOT, "profiles", "correlation")
    try:
        p = os.path.join(cdir, open(os.path.join(cdir, "LATEST")).read().strip())
    except OSError:
        runs = sorted(f for f in os.listdir(cdir) if f.endswith("_gpu.json")) if os.path.isdir(cdir) else []
        p = os.path.join(cdir, runs[-1]) if runs else ""
    try:
        d = json.load(open(p))["Cycles"]
        cfg, v = next(iter(d.items()))
        return {"mae_pct": round(v["app_incl_noisy"]["mae"], 2), "apps": v["app_incl_noisy"]["n"],
                "mae_pct_stable_apps": round(v["app"]["mae"], 2), "stable_apps": v["app"]["n"],
                "pearson": round(v["app_incl_noisy"]["correl"], 4), "gpu": "MI355X", "config": cfg,
                "traces": "automatic gfx950 ISA traces (isatrace)", "measured": "offline, not in this run",
                "engine": "cpu (bit-exact with the GPU engine)" if "local" in os.path.basename(p) else "gpu",
                "protocol": "every config parameter from micro-benchmarks (tools/gpu_correlate.sh tuner); HW "
                            "cycles the mean of 4 rocprofv3 runs",
                "source": os.path.relpath(p, ROOT)}
    except (OSError, ValueError, KeyError, StopIteration):
        return None


def _cfg_desc(name: str) -> str:
    return {"GV100": "SM7_GV100 gpgpusim.config = SM7_QV100 at 1447 MHz, + SM7_QV100 trace.config",
            "QV100": "SM7_QV100 gpgpusim.config + trace.config"}.get(name, "preset " + name)


def _resolve_app(rodinia, name: str) -> str:
    """Full suite name for `name` ("nw" -> "nw-rodinia-2.0-ft"); unknown names fail.
    "dp-step" selects the data-parallel training step."""
    if name in rodinia.SUITE or name == "dp-step":
        return name
    hit = [k for k in rodinia.SUITE if k.split("-rodinia")[0] == name]
    if not hit:
        raise SystemExit(f"bench.py: unknown app {name!r}; known: {', '.join(rodinia.SUITE)}")
    return hit[0]


def _sweep(a, suite, engine, rank, world, use_cuda) -> int:
    """``--sweep``: the tuner's configuration sweep as the step (one batch of
    apps x 16 configs per rank, weak scaling over ranks)."""
    import torch
    from accel_sim_framework_distributed_amd.parallel.sweep import SweepRunner
    run = SweepRunner(suite, a.sweep_configs)

    def sync():
        if use_cuda:
            torch.cuda.synchronize()
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    ratio = run.calibrate()  # node: untimed GPU/CPU ratio per app (queue order)
    for _ in range(a.warmup):
        run.step()
    sync()
    t0 = time.perf_counter()
    insn = insn_gpu = jobs_gpu = jobs_cpu = 0
    for _ in range(a.steps):
        r = run.step()
        insn += r["insn"]
        insn_gpu += r["insn_gpu"]
        jobs_gpu += r["jobs_gpu"]
        jobs_cpu += r["jobs_cpu"]
    sync()
    dt = time.perf_counter() - t0
    mine = {"rank": rank, "wall_s": round(dt, 4), "insn": int(insn), "insn_gpu": int(insn_gpu),
            "jobs_gpu": jobs_gpu, "jobs_cpu": jobs_cpu}
    per_rank = suite.gather(mine)
    dt_max = max(p["wall_s"] for p in per_rank)
    insn_all = sum(p["insn"] for p in per_rank)
    gpu_all = sum(p["insn_gpu"] for p in per_rank)
    kips = insn_all / max(dt_max, 1e-9) / 1e3
    if rank == 0:
        out = {
            "metric": "sim KIPS (whole node), tuner config sweep",
            "value": round(kips, 3),
            "unit": "KIPS (thousand simulated thread-instructions / wall s, summed over ranks)",
            "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(dt_max / max(1, a.steps) * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": round(kips / BASELINE_KIPS, 3),
            "vs_baseline_note": "not like-for-like: reference = GPGPU-Sim, 1 CPU core, recorded heartwall traces",
            "vs_baseline_parts": _baseline_parts(kips, gpu_all / max(dt_max, 1e-9) / 1e3, suite, engine, world),
            "dtype": "n/a (integer cycle-level model)",
            "data": "synthetic (seeded Rodinia-2.0-ft-shaped SASS traces)",
            "config": {"model": f"{a.config} ({_cfg_desc(a.config)}), BASELINE config #5 shape: "
                                f"{len(run.jobs) // max(1, len(run.configs))} apps x {len(run.configs)} tuner "
                                "search configs (scheduler x L2 granularity x hash x DRAM scheduler)",
                       "global_batch": world, "seq_len": None,
                       "parallelism": f"job-level: GPU-engine CU groups + host cores per rank (dp{world})",
                       "engine": engine, "jobs_per_step_per_rank": len(run.jobs),
                       "configs": [c for c, _ in run.configs],
                       "gpu_slots": run.last.get("gpu_slots"), "cpu_slots": run.last.get("cpu_slots"),
                       "gpu_over_cpu_time_ratio": {k: round(v, 3) for k, v in ratio.items()}},
            "gpu_engine": {"kips_whole_node": round(gpu_all / max(dt_max, 1e-9) / 1e3, 1),
                           "insn_share": round(gpu_all / max(insn_all, 1), 4),
                           "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0),
                           "jobs": sum(p["jobs_gpu"] for p in per_rank)},
            "cpu_engine": {"kips_whole_node": round((insn_all - gpu_all) / max(dt_max, 1e-9) / 1e3, 1),
                           "jobs": sum(p["jobs_cpu"] for p in per_rank)},
            "per_rank": per_rank,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


def _baseline_parts(kips, gpu_kips, suite, engine, world):
    """The headline split into what the MI355X cycle engine simulated and what
    the host cores did, each against the reference's one-core 349 KIPS."""
    cores = suite.cpu_slots(reserve=suite.gpu_reserve(max(1, suite.concurrency()))) if engine in ("node", "cpu") else 0
    host = max(0.0, kips - gpu_kips)
    per_core = host / max(1, cores * world) if cores else 0.0
    return {"gpu_engine_kips": round(gpu_kips, 1), "gpu_engine_vs_baseline": round(gpu_kips / BASELINE_KIPS, 3),
            "host_kips": round(host, 1), "host_cores": cores * world,
            "host_kips_per_core": round(per_core, 1), "host_per_core_vs_baseline": round(per_core / BASELINE_KIPS, 3)}


def main() -> int:
    a = _parse()
    _gpu_env(bool(a.sweep))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    use_cuda = torch.cuda.is_available()
    if use_cuda:
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = a.dist_backend if a.dist_backend != "auto" else ("nccl" if use_cuda else "gloo")
        dist.init_process_group(backend)
    # collective operands live where the backend reads them
    on_dev = use_cuda and (world == 1 or dist.get_backend() == "nccl")
    dev = torch.device("cuda", torch.cuda.current_device()) if on_dev else torch.device("cpu")

    from accel_sim_framework_distributed_amd import _native
    mod = _native.load(prefer_torch_runtime=True)
    engine = a.engine
    if engine == "auto":
        engine = "node" if mod.gpu_available() else "cpu"
    mock = os.environ.get("ASIM_MOCK_GPU", "0") not in ("", "0")  # CPU-tier rehearsal (multi_gpu.mock_gpu)
    if engine in ("gpu", "node") and not mod.gpu_available() and not mock:
        raise SystemExit(f"bench.py: --engine {engine} requested but no HIP device is usable")

    from accel_sim_framework_distributed_amd.parallel.multi_gpu import DistributedSuite
    from accel_sim_framework_distributed_amd.tracegen import rodinia

    tdir = a.trace_dir or os.path.join(tempfile.gettempdir(),
                                       f"asim_bench_rodinia_v{rodinia.SUITE_VERSION}_{os.getuid()}")
    apps = None if a.apps == "all" else [_resolve_app(rodinia, x) for x in a.apps.split(",")]
    # every rank generates (or reuses) the deterministic synthetic traces
    # a generated subset never stands in for the full suite (and vice versa is fine)
    full_marker = os.path.join(tdir, ".complete-all")
    marker = full_marker if apps is None else os.path.join(tdir, ".complete-" + "+".join(sorted(apps))[:200])
    if apps is not None and os.path.exists(full_marker):
        marker = full_marker
    # the all-reduce example is traced per rank count, so a cached suite from a
    # run with another GPU count never hands this run a collective of the
    # wrong size (which the simulator would then emulate locally)
    ar_dir = os.path.join(tdir, f"all-reduce-{max(1, world)}")
    ar_marker = os.path.join(ar_dir, ".complete")
    # the step's data-parallel training trace, one per rank (unequal shards:
    # rank r computes 1 + 0.25 r/(N-1) of the base batch, so the per-layer
    # gradient all-reduces couple the ranks' simulated clocks)
    dp_dir = os.path.join(tdir, f"dp-step-{max(1, world)}")
    dp_marker = os.path.join(dp_dir, ".complete")
    if rank == 0:
        os.makedirs(tdir, exist_ok=True)
        if not os.path.exists(marker):
            rodinia.generate_suite(tdir, apps)
            open(marker, "w").write("ok")
        if not os.path.exists(ar_marker):
            rodinia.write_allreduce_example(ar_dir, nranks=max(1, world))
            open(ar_marker, "w").write("ok")
        if not os.path.exists(dp_marker):
            from accel_sim_framework_distributed_amd.tracegen import training
            training.write_dp_ranks(dp_dir, max(1, world), straggle=0.25)
            open(dp_marker, "w").write("ok")
    if world > 1:
        dist.barrier()
    while not (os.path.exists(marker) and os.path.exists(ar_marker) and os.path.exists(dp_marker)):
        time.sleep(0.1)

    suite = DistributedSuite(tdir, config=a.config, engine=engine, rank=rank, world=world, apps=apps,
                             verbose=a.verbose and rank == 0)
    if a.sweep:
        return _sweep(a, suite, engine, rank, world, use_cuda)

    def sync():
        if use_cuda:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    if engine == "node":
        # untimed: time every application on both engines, then place them
        suite.calibrate()
        # host threads for the CPU-engine applications on the critical path
        # (spare cores only; each app's team is re-timed before it is kept)
        suite.widen()
        suite.plan()
    # one plan for the whole job: every rank runs rank 0's placement (ranks
    # calibrate under their own host load and could otherwise disagree)
    own_plan_matched = suite.agree_plan() if engine == "node" else True
    for _ in range(a.warmup):
        suite.step()
    sync()
    t0 = time.perf_counter()
    insn = 0
    insn_gpu = 0
    cycles = 0
    last_apps = {}
    for _ in range(a.steps):
        r = suite.step()
        last_apps = r.get("apps", {})
        insn += r["insn"]
        insn_gpu += r["insn_gpu"]
        cycles += r["cycles"]
    sync()
    dt = time.perf_counter() - t0
    # max wall time over ranks, total instructions over ranks; the DDP step's
    # simulated cycles: max over ranks (the step ends with the slowest rank)
    dpl = suite.dp_last or {}
    t = torch.tensor([dt, float(insn), float(cycles), float(dpl.get("cycles", 0)), float(insn_gpu)],
                     dtype=torch.float64, device=dev)
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        dt, insn_all, cyc_all, dp_max = float(tmax[0]), float(tsum[1]), float(tsum[2]), float(tmax[3])
        gpu_all = float(tsum[4])
        # every rank's GPU-engine share (all_gather: the bench prints per-rank values)
        g = torch.zeros(world, dtype=torch.float64, device=dev)
        g[rank] = float(insn_gpu) / max(dt, 1e-9) / 1e3
        dist.all_reduce(g, op=dist.ReduceOp.SUM)
        gpu_per_rank = [round(float(x), 1) for x in g.cpu()]
        dc = torch.zeros(world, dtype=torch.float64, device=dev)
        dc[rank] = float(dpl.get("cycles", 0))
        dist.all_reduce(dc, op=dist.ReduceOp.SUM)
        dp_cycles_per_rank = [int(x) for x in dc.cpu()]
    else:
        insn_all, cyc_all, dp_max = float(insn), float(cycles), float(dpl.get("cycles", 0))
        gpu_all = float(insn_gpu)
        gpu_per_rank = [round(gpu_all / dt / 1e3, 1)]
        dp_cycles_per_rank = [int(dpl.get("cycles", 0))]
    kips = insn_all / dt / 1e3
    # every rank's own view (gathered to all; rank 0 prints it)
    mine = {"rank": rank, "wall_s": round(dt, 4), "insn": int(insn), "insn_gpu": int(insn_gpu),
            "kips": round(insn / max(dt, 1e-9) / 1e3, 1),
            "gpu_insn_share": round(insn_gpu / max(insn, 1), 4)}
    if engine == "node":
        mine.update(assignment=suite.assignment, cpu_threads={k: v for k, v in suite.threads.items() if v > 1},
                    calibration_s=suite.calibration, own_plan_matched_rank0=bool(own_plan_matched),
                    plan_source=suite.plan_source)
    per_rank = suite.gather(mine)
    plans_identical = all(p.get("assignment") == per_rank[0].get("assignment") and
                          p.get("cpu_threads") == per_rank[0].get("cpu_threads") for p in per_rank)
    walls = [p["wall_s"] for p in per_rank]
    if rank == 0:
        out = {
            "metric": "sim KIPS (whole node)",
            "value": round(kips, 3),
            "unit": "KIPS (thousand simulated thread-instructions / wall s, summed over ranks)",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / max(1, a.steps) * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(kips / BASELINE_KIPS, 3),
            # not like-for-like: the baseline is GPGPU-Sim on one CPU core on
            # recorded QV100 heartwall traces (util/job_launching/README.md:77);
            # this run is this simulator on synthetic suite-shaped traces
            "vs_baseline_note": "not like-for-like: reference = GPGPU-Sim, 1 CPU core, recorded heartwall "
                                "traces (349 KIPS); this = MI355X-native simulator, synthetic Rodinia-2.0-ft-"
                                "shaped traces, engine placement in config.engine",
            # the ratio above divides a whole node (host cores + MI355X) by one
            # reference core; its parts, each against the same 349 KIPS:
            "vs_baseline_parts": _baseline_parts(kips, gpu_all / dt / 1e3, suite, engine, world),
            "dtype": "n/a (integer cycle-level model)",
            "data": "synthetic (seeded Rodinia-2.0-ft-shaped SASS traces; no recorded traces available)",
            "config": {
                "model": f"{a.config} ({_cfg_desc(a.config)}) simulating rodinia_2.0-ft",
                "global_batch": world,
                "seq_len": None,
                "parallelism": f"one simulated GPU per MI355X rank (dp{world}), RCCL-synchronised collectives",
                "engine": engine,
                **({"node_assignment": suite.assignment,
                    "node_calibration_s": suite.calibration,
                    "node_predicted_step_ms": round(suite.predicted_span * 1e3, 1),
                    "node_cpu_threads": {k: v for k, v in suite.threads.items() if v > 1},
                    # wall seconds of every application in the last timed step
                    # (the step's makespan is the longest of them)
                    "node_step_wall_s": {k: round(v.get("wall_s", 0.0), 4) for k, v in last_apps.items()},
                    "node_host_cores": suite.cpu_slots(reserve=suite.gpu_reserve(max(1, suite.concurrency())))} if engine == "node" else {}),
                "apps": len(suite.apps),
                "sim_insn_per_step_per_rank": int(insn / max(1, a.steps)),
                "sim_cycles_per_step_per_rank": int(cycles / max(1, a.steps)),
            },
            # the part of the headline simulated by the HIP cycle engine on the
            # MI355X(s): thread instructions of the applications the GPU engine
            # ran, over the same wall time (the rest ran on host cores)
            "gpu_engine": {"kips_whole_node": round(gpu_all / dt / 1e3, 1),
                           "kips_per_rank": gpu_per_rank,
                           "insn_share": round(gpu_all / max(insn_all, 1.0), 4),
                           "apps_on_gpu": (sum(1 for v in suite.assignment.values() if v == "gpu")
                                           if engine == "node" else (len(suite.apps) if engine == "gpu" else 0)),
                           "apps": len(suite.apps),
                           "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0)},
            "per_rank": per_rank,
            "plans_identical": plans_identical,
            "wall_s_spread": {"min": min(walls), "max": max(walls)},
            "cycle_mae_vs_hw": _cycle_mae(),
            "dp_step": ({"ranks": world, "simulated_cycles_max_rank": int(dp_max),
                         "simulated_cycles_per_rank": dp_cycles_per_rank,
                         "collective_mem_traffic": True,
                         "rank0_kernels": dpl.get("kernels"), "rank0_collectives": dpl.get("collectives"),
                         "rank0_comm_cycles": dpl.get("comm_cycles"),
                         "collective_coupling": dpl.get("modes"),
                         "streams": "per-layer gradient all-reduce on stream 2 overlapping backward on stream 1"}
                        if dpl else None),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
